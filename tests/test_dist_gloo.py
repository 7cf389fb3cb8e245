"""Multi-process (world_size 2, gloo, CPU) tests of the replicate-sharding path:
disjoint covering shards, accumulator all-gather and rank-ordered deterministic merge."""
import ctypes as C
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_covers_disjointly():
    from dcor.dist import shard
    for B in (1, 7, 250, 1000, 100_003):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard(B, r, world) for r in range(world)]
            pos = 0
            for b0, nb in ranges:
                assert b0 == pos and nb >= 0
                pos += nb
            assert pos == B
            assert max(nb for _, nb in ranges) - min(nb for _, nb in ranges) <= 1


def _fake_accums(rank, ncells):
    from dcor import _lib
    g = np.random.default_rng(100 + rank)
    out = []
    for i in range(2 * ncells):
        a = _lib.Accum()
        a.n = 10 + rank
        a.n_cover = int(g.integers(0, 10))
        for f in ("est", "est2", "se2", "len", "lo", "hi"):
            getattr(a, f)[0] = float(g.normal())
        out.append(a)
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcor.dist import gather_accums, merge_ranked
    local = _fake_accums(rank, 3)
    per_rank = gather_accums(local)
    merged = merge_ranked(per_rank)
    q.put((rank, [bytes(a) for a in merged]))
    dist.destroy_process_group()


def test_gather_merge_two_ranks():
    from dcor import _lib
    from dcor.sim import merge
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # identical on both ranks, and equal to the rank-ordered merge done locally
    assert res[0] == res[1]
    want = [merge([_fake_accums(r, 3)[i] for r in range(world)]) for i in range(6)]
    assert res[0] == [bytes(a) for a in want]
    a0 = _lib.Accum.from_buffer_copy(res[0][0])
    assert a0.n == 10 + 11


def test_rstream_cell_shard_balanced_and_covering():
    from dcor.dist import cell_shard
    g = np.random.default_rng(3)
    for ncells in (1, 5, 144, 480):
        costs = list(g.choice([1e3, 1e4, 1e5, 1e6], ncells) * 250.0)
        for world in (1, 2, 4, 8):
            parts = cell_shard(costs, world)
            flat = sorted(i for p in parts for i in p)
            assert flat == list(range(ncells))
            loads = [sum(costs[i] for i in p) for p in parts]
            # LPT: the heaviest rank exceeds the lightest by at most one cell's cost
            assert max(loads) - min(loads) <= max(costs) + 1e-9
            assert parts == cell_shard(costs, world)  # deterministic


def _rs_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcor import _lib
    from dcor.dist import cell_shard, gather_accums, merge_ranked
    # cell i's accumulators exist only on its owner; the merge must reproduce them exactly
    costs = [1.0, 5.0, 2.0, 2.0, 7.0]
    mine = cell_shard(costs, world)[rank]
    local = [_lib.Accum() for _ in range(2 * len(costs))]
    for i in mine:
        for m in range(2):
            a = _lib.Accum()
            a.n = 100 + 10 * i + m
            a.est[0] = 0.125 * (i + 1) + m
            a.est[1] = 1e-20 * (i + 1)
            local[2 * i + m] = a
    merged = merge_ranked(gather_accums(local))
    q.put((rank, [(a.n, a.est[0], a.est[1]) for a in merged]))
    dist.destroy_process_group()


def test_rstream_cell_shard_gather_two_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rs_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    for i in range(5):
        for m in range(2):
            assert res[0][2 * i + m] == (100 + 10 * i + m, 0.125 * (i + 1) + m, 1e-20 * (i + 1))


def test_sweep_shard_covers_flattened_space():
    from dcor.dist import shard, sweep_shard
    for n_eps, reps in ((23, 200), (3, 7), (1, 1), (5, 1)):
        for world in (1, 2, 3, 8, 13):
            seen = []
            for r in range(world):
                segs = sweep_shard(n_eps, reps, r, world)
                assert sum(c for _, _, c in segs) == shard(n_eps * reps, r, world)[1]
                for e, r0, c in segs:
                    assert 0 <= e < n_eps and 0 <= r0 and c >= 1 and r0 + c <= reps
                    seen.extend(e * reps + r0 + i for i in range(c))
            assert seen == list(range(n_eps * reps))   # rank order = flattened order


def _rows_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dcor.dist import gather_rows, shard
    total = 11
    counts = [shard(total, r, world)[1] for r in range(world)]
    b0, nb = shard(total, rank, world)
    local = np.arange(b0 * 6, (b0 + nb) * 6, dtype=np.float64).reshape(nb, 6) + 0.5
    q.put((rank, gather_rows(local, counts).tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_ranks_in_order(world):
    """dcor.dist.gather_rows (the HRS records' all-gather): uneven shards padded to the largest and
    trimmed, concatenated in rank order, identical on every rank."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = (np.arange(11 * 6, dtype=np.float64).reshape(11, 6) + 0.5).tobytes()
    assert all(v == want for v in res.values())
