"""CPU tests of bench.py's launcher (VERDICT r03 "next" #2): `--gpus N` without torchrun starts N
rank processes that form one process group, and a mismatch between --gpus and a launcher's
WORLD_SIZE is refused, so a multi-GPU run can never silently measure one GPU
(vert-cor.R:513,534-553 is the mclapply fan-out this replaces)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=180, env=e)


def test_gpus_2_spawns_two_ranks():
    p = _run(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout              # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_formed"] == 2
    assert d["merged_n"] == 1 + 2                 # both ranks' accumulators, merged in rank order
    assert d["value"] is None                     # a dry run measures nothing


def test_gpus_3_spawns_three_ranks():
    p = _run(["--gpus", "3", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 3 and d["merged_n"] == 6


def test_gpus_mismatch_with_launcher_is_refused():
    p = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def test_more_gpus_than_visible_is_refused():
    p = _run(["--gpus", "2", "--no-cpu-baseline"], env={"HIP_VISIBLE_DEVICES": ""})
    assert p.returncode != 0
    assert "visible" in p.stderr


def test_failing_rank_stops_the_others():
    """A rank that dies before the rendezvous must not leave the other ranks waiting in it: the
    launcher stops them and exits non-zero, promptly."""
    import time
    t0 = time.time()
    p = _run(["--gpus", "2", "--dry-run"], env={"DCOR_BENCH_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert time.time() - t0 < 120


def test_launcher_parent_loads_no_gpu_library():
    """`--gpus N` spawns its ranks before anything GPU-side is imported: at the spawn the parent has
    neither torch nor amdsmi in sys.modules; the ranks check their devices."""
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "def spawn(n, argv):\n"
            "    bad = [m for m in ('torch', 'torch.cuda', 'amdsmi') if m in sys.modules]\n"
            "    print('LOADED' if bad else 'CLEAN', bad)\n"
            "    return 0\n"
            "bench.spawn_ranks = spawn\n"
            "sys.argv = ['bench.py', '--gpus', '4', '--no-cpu-baseline']\n"
            "bench.main()\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "CLEAN" in p.stdout, p.stdout


def _run_configs(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench_configs.py")] + args, capture_output=True,
                          text=True, timeout=180, env=e)


def test_configs_gpus_2_forms_two_ranks_for_c3_c4():
    """bench_configs.py --gpus 2: two rank processes form one group and
    split every C3 / C4 cell's replicates into contiguous shards (vert-cor.R:513,534-553)."""
    p = _run_configs(["--gpus", "2", "--dry-run", "--only", "C3,C4"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert [d["config"] for d in lines] == ["C3", "C4"]     # rank 0 only
    c3, c4 = lines
    assert c3["world_formed"] == 2 and c3["replicates"] == 24 * 100_000
    assert c3["shards"] == [[[0, 50_000], [50_000, 50_000]]]
    assert c4["world_formed"] == 2 and c4["shards"][1] == [[0, 50_000], [50_000, 50_000]]


def test_configs_gpus_2_forms_two_ranks_for_hrs():
    """The HRS workload shards too: C5 weak (each rank its own 8192-replicate
    range), C5-e2e / C5-fused over contiguous ranges of 1e6 replicates, the eps sweep over the
    flattened (eps, run) space (real-data-sims.R:411-436)."""
    p = _run_configs(["--gpus", "2", "--dry-run", "--only", "C5,C5e,C5f,C5fc,HS"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = {d["config"]: d for d in (json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{"))}
    assert set(lines) == {"C5", "C5-e2e", "C5-fused", "C5-fused-continuous", "HS"}
    assert all(d["world_formed"] == 2 for d in lines.values())
    assert lines["C5"]["shards"] == [[0, 8192], [8192, 8192]]
    assert lines["C5-e2e"]["shards"] == [[0, 500_000], [500_000, 500_000]]
    hs = lines["HS"]
    assert hs["replicates"] == 23 * 200
    assert sum(c for segs in hs["shards"] for _, _, c in segs) == 4600
    assert hs["shards"][1][0] == [11, 100, 100]


def test_configs_more_gpus_than_visible_is_refused():
    p = _run_configs(["--gpus", "2", "--only", "C3"], env={"HIP_VISIBLE_DEVICES": ""})
    assert p.returncode != 0
    assert "visible" in p.stderr


def test_config_lines_physical_fractions_from_timed_kernels():
    """bench_configs.measured(): each config line names its committed profile, whether that profile
    was taken on this tree's engine sources, and per-kernel physical fractions; VG and SG, whose
    profiles also hold the per-cell comparison loop, report the timed grid call's kernels only."""
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    bc = importlib.import_module("bench_configs")
    for name in ("VG", "SG", "C3", "C5-continuous"):
        m = bc.measured(name)
        assert m and m["profile"].startswith("profiles/") and isinstance(m["profile_fresh"], bool)
        assert m["physical"], name
        for k, v in m["physical"].items():
            assert v["pct_time"] >= 5.0
            if name in bc.TIMED_KERNELS:
                assert k.startswith(bc.TIMED_KERNELS[name]), (name, k)
    assert bc.measured("C1") == {}
