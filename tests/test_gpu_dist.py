"""GPU tests of the replicate-sharding path (dcor.dist; replaces mclapply over cells,
vert-cor.R:534-553): the RCCL all-gather at world size 1 on this box's one GPU, and two
ranks sharing cuda:0 over gloo -- each rank simulates its shard on the GPU, the merged
summaries equal the rank-ordered merge of the same shards computed in one process."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B = 37  # odd: the two shards differ in size


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cells():
    from dcor.sim import CellSpec, headline_cell
    return [headline_cell(5000),
            CellSpec(n=3001, rho=0.65, eps1=1.5, eps2=0.5, family="subG", dgp="bounded_factor", seed=1_000_007),
            CellSpec(n=2000, rho=0.3, eps1=1.0, eps2=1.0, family="sign", dgp="bernoulli", seed=1_000_008)]


def _expected(world):
    """Per-rank shard accumulators computed in this process, merged in rank order."""
    from dcor.dist import merge_ranked, shard
    from dcor.sim import accum_from_bytes, accumulate, simulate
    per_rank = []
    for r in range(world):
        b0, nb = shard(B, r, world)
        local = []
        for cell in _cells():
            out = simulate(cell, nb, b0)
            local.extend(accum_from_bytes(accumulate(out, cell.rho).cpu().numpy().tobytes()))
        per_rank.append(local)
    return [bytes(a) for a in merge_ranked(per_rank)]


def _flat(merged):
    return [bytes(a) for pair in merged for a in pair]


def test_run_grid_distributed_rccl_world1():
    import torch
    import torch.distributed as dist
    from dcor.dist import run_grid_distributed
    assert torch.cuda.is_available()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        got = _flat(run_grid_distributed(_cells(), B))
    finally:
        dist.destroy_process_group()
    assert got == _expected(1)
    _assert_equals_world1(got)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcor.dist import run_grid_distributed
    pairs, (b0, rec) = run_grid_distributed(_cells(), B, return_records=True)
    q.put((rank, (_flat(pairs), b0, rec.tobytes(), rec.shape)))
    dist.destroy_process_group()


def test_run_grid_distributed_two_ranks_on_gpu():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    res = {r: v[0] for r, v in got.items()}
    assert res[0] == res[1]
    assert res[0] == _expected(world)
    _assert_equals_world1(res[0])
    # the batched shards' replicates, concatenated in rank order, are the world-1 run's bit for bit
    import numpy as np
    from dcor.sim import simulate
    parts = [np.frombuffer(got[r][2], dtype=np.float64).reshape(got[r][3]) for r in range(world)]
    assert [got[r][1] for r in range(world)] == [0, B // 2]
    for i, cell in enumerate(_cells()):
        want = simulate(cell, B, 0).cpu().numpy()
        have = np.concatenate([p[i] for p in parts])
        assert np.array_equal(have.view(np.uint64), want.view(np.uint64)), cell


def _world1():
    """The unsharded run: every replicate of each cell in one launch, one accumulation."""
    from dcor.sim import accum_from_bytes, accumulate, simulate
    out = []
    for cell in _cells():
        rec = simulate(cell, B, 0)
        out.extend(accum_from_bytes(accumulate(rec, cell.rho).cpu().numpy().tobytes()))
    return out


def _assert_equals_world1(flat):
    """Merged world-2 accumulators vs the world-1 run: counts exactly, every double-double sum
    within 1e-15 relative, and the finalized summaries (mse, bias, var, coverage, ci_length;
    vert-cor.R:422-430) within 1e-13 relative -- bias and var cancel (mean - rho,
    E[x^2] - E[x]^2), which magnifies the sums' last-bit differences."""
    import math

    from dcor import _lib
    from dcor.sim import finalize
    ref = _world1()
    cells = _cells()
    for i, (raw, r) in enumerate(zip(flat, ref)):
        a = _lib.Accum.from_buffer_copy(raw)
        for f in ("n", "n_cover", "n_cover_na", "n_na_est", "n_na_ci"):
            assert getattr(a, f) == getattr(r, f), (i, f)
        for f in ("est", "est2", "se2", "len", "lo", "hi"):
            x, y = getattr(a, f)[0] + getattr(a, f)[1], getattr(r, f)[0] + getattr(r, f)[1]
            assert abs(x - y) <= 1e-15 * max(abs(x), abs(y), 1e-300) or x == y, (i, f, x, y)
        rho = cells[i // 2].rho
        sa, sr = finalize(a, rho), finalize(r, rho)
        for k in sa:
            x, y = sa[k], sr[k]
            assert (math.isnan(x) and math.isnan(y)) or abs(x - y) <= 1e-13 * max(abs(x), abs(y)) + 1e-300, (i, k, x, y)


def test_bench_configs_c3_over_ranks_runs():
    """bench_configs.py --gpus 1 takes the rank path C3 / C4 use on a node (one process per GPU,
    RCCL all-gather of the accumulators) and prints a measured line with the world it formed; a
    reduced C3 (64 replicates per cell of the eps = (1, 1) cells)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench_configs.py"), "--gpus", "1", "--only", "C3",
                        "--c3-reps", "64", "--c3-eps", "1x1"], capture_output=True, text=True, timeout=240, env=e)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["config"] == "C3" and d["world_formed"] == 1 and d["backend"] == "nccl"
    assert d["replicates"] == 8 * 64 and d["cells_with_results"] == 8 and d["reps_per_s"] > 0


# ------------------------------------------------ the HRS workload over ranks (a19 / C5)
HRS_R = 41          # odd: uneven shards
SWEEP = (0.55, 1.35, 2.05)


def _hrs_args():
    import numpy as np
    from dcor import hrs
    age, bmi = hrs.standin_panel(3001, -0.3, seed=5)
    z = hrs.standardize_panel(age, bmi, lap=np.array([0.3, -0.2, 0.1, 0.4]))
    return (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"])


def _hrs_runs():
    """[premat, fused, R-stream] records of HRS_R replicates, and the sweep's runs + summaries."""
    from dcor.dist import eps_sweep_distributed, run_hrs_distributed
    a = _hrs_args()
    recs = [run_hrs_distributed(*a, 2.0, HRS_R, rep_begin=3),
            run_hrs_distributed(*a, 2.0, HRS_R, rep_begin=3, mode="fused"),
            run_hrs_distributed(*a, 0.75, 9, rng="R", eps_idx=6)]
    sw = eps_sweep_distributed(*a, eps_grid=SWEEP, reps=7)
    return [r.tobytes() for r in recs], sw["runs"].tobytes(), sw["ni_mean"], sw["int_mean"]


def _hrs_expected():
    from dcor import hrs
    a = _hrs_args()
    recs = [hrs.hrs_replicates(*a, 2.0, HRS_R, rep_begin=3),
            hrs.hrs_replicates(*a, 2.0, HRS_R, rep_begin=3, mode="fused"),
            hrs.hrs_replicates(*a, 0.75, 9, rng="R", eps_idx=6)]
    sw = hrs.eps_sweep(*a, eps_grid=SWEEP, reps=7)
    return [r.tobytes() for r in recs], sw["runs"].tobytes(), sw["ni_mean"], sw["int_mean"]


def test_hrs_distributed_rccl_world1():
    """dcor.dist.run_hrs_distributed / eps_sweep_distributed at world 1 over RCCL: the records
    equal one process's hrs_replicates byte for byte, the sweep equals eps_sweep."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        got = _hrs_runs()
    finally:
        dist.destroy_process_group()
    assert got == _hrs_expected()


def _hrs_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q.put((rank, _hrs_runs()))
    dist.destroy_process_group()


def test_hrs_distributed_two_ranks_on_gpu():
    """Two gloo ranks sharing cuda:0: each runs its contiguous replicate range (and its part of the
    flattened sweep); the gathered records are the single-process run's byte for byte on both."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hrs_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    want = _hrs_expected()
    assert got[0] == want and got[1] == want


def test_bench_configs_hrs_over_ranks_runs():
    """bench_configs.py --gpus 1 --only C5e,HS takes the HRS rank path and prints lines with the
    world it formed (reduced sizes)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench_configs.py"), "--gpus", "1", "--only",
                        "C5,C5e,HS", "--c5-R", "512", "--c5e-R", "3000", "--hs-R", "20"], capture_output=True,
                       text=True, timeout=240, env=e)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = {d["config"]: d for d in (json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{"))}
    assert lines["C5-e2e"]["world_formed"] == 1 and lines["C5-e2e"]["rows_gathered"] == 3000
    assert lines["HS"]["rows_gathered"] == 23 * 20 and lines["HS"]["finite"]
    assert lines["C5"]["replicates"] == 512 and lines["C5"]["reps_per_s"] > 0
