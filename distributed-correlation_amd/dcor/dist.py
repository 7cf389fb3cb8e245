"""Multi-GPU replicate sharding (one process per GPU, torch.distributed over RCCL).

The path shards with no data-path collective: for every cell, rank g of G runs the
contiguous replicate range [g*B/G, (g+1)*B/G) (counter-based RNG: a replicate's
numbers depend only on (seed, rep)).  The only exchange is the per-(cell, method)
summary accumulators -- 160 B each -- gathered once per grid and merged in rank order,
so the merged summary is deterministic for a given G (double-double sums).
Replaces parallel::mclapply over cells (vert-cor.R:534-553; ver-cor-subG.R:294-295).
"""
from __future__ import annotations

import ctypes as C
from typing import List

import numpy as np

from . import _lib

ACC_BYTES = C.sizeof(_lib.Accum)


def shard(B: int, rank: int, world: int):
    """Contiguous replicate range of `rank`: (begin, count)."""
    b0 = B * rank // world
    b1 = B * (rank + 1) // world
    return b0, b1 - b0


def gather_accums(local: List[_lib.Accum], group=None) -> List[List[_lib.Accum]]:
    """All-gather a list of accumulators from every rank -> [rank][i] (host objects).

    Uses the process group's backend (RCCL when 'nccl', gloo on CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    raw = b"".join(bytes(a) for a in local)
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).clone()
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    per_rank = []
    for o in outs:
        b = o.cpu().numpy().tobytes()
        per_rank.append([_lib.Accum.from_buffer_copy(b[i * ACC_BYTES:(i + 1) * ACC_BYTES])
                         for i in range(len(local))])
    return per_rank


def merge_ranked(per_rank: List[List[_lib.Accum]]) -> List[_lib.Accum]:
    """Merge accumulator i over ranks in rank order (deterministic)."""
    from .sim import merge
    n = len(per_rank[0])
    return [merge([per_rank[r][i] for r in range(len(per_rank))]) for i in range(n)]


def run_grid_distributed(cells, B: int, group=None, stream=None, return_records: bool = False):
    """Every rank runs its replicate shard [g B / G, (g+1) B / G) of EVERY cell in one batched
    launch sequence (dcor_grid_launch: all cells' replicates share the launches, so a rank's few
    replicates per cell still fill its GPU), then the per-cell accumulators are all-gathered --
    straight from device memory under RCCL -- copied to the host once and merged in rank order.
    Returns [(NI, INT)] per cell, identical on all ranks; with return_records also this rank's
    (b0, records [ncells, nb, 6]) (byte-identical to the same replicates of a world-1 run)."""
    import torch
    import torch.distributed as dist

    from .sim import grid_launch

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    b0, nb = shard(B, rank, world)
    nc = len(cells)
    s = torch.cuda.current_stream() if stream is None else stream
    with torch.cuda.stream(s):   # torch's copies and the collective's device work run on `s`
        if nb > 0:
            out, acc = grid_launch(cells, b0, nb, stream=s)
        else:
            out = None
            acc = torch.zeros(2 * nc * ACC_BYTES, dtype=torch.uint8, device="cuda")
        t = acc if dist.get_backend(group) == "nccl" else acc.cpu()
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        raw = torch.cat(outs).cpu().numpy().tobytes()          # the one D2H copy
        rec = out.cpu().numpy().reshape(nc, nb, 6) if (return_records and out is not None) else None
    per_rank = [[_lib.Accum.from_buffer_copy(raw[(r * 2 * nc + i) * ACC_BYTES:(r * 2 * nc + i + 1) * ACC_BYTES])
                 for i in range(2 * nc)] for r in range(world)]
    merged = merge_ranked(per_rank)
    pairs = [(merged[2 * i], merged[2 * i + 1]) for i in range(nc)]
    if return_records:
        return pairs, (b0, rec if rec is not None else np.zeros((nc, 0, 6)))
    return pairs


# ------------------------------------------------------ R-stream mode (by cell)
def cell_shard(costs, world: int) -> List[List[int]]:
    """Cells of an R-stream grid per rank.  R's stream is sequential within a cell, so the cell
    is the unit (the reference's mclapply unit); longest-processing-time-first on cost (n * B),
    ties by cell index, deterministic for a given world size."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        g = min(range(world), key=lambda r: (load[r], r))
        out[g].append(i)
        load[g] += costs[i]
    return [sorted(o) for o in out]


def run_grid_rstream_distributed(cells, B: int, group=None):
    """R-stream grid over G ranks: rank g runs its cells of cell_shard() with R's own streams
    (dcor.rstream); the per-cell accumulators are all-gathered (cells a rank does not own
    contribute empty accumulators) and merged in rank order.  Returns [(NI, INT)] per cell,
    identical on all ranks and equal to a single-GPU run."""
    import torch.distributed as dist

    from .rstream import run_grid

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mine = cell_shard([float(c.n) * B for c in cells], world)[rank]
    local = [_lib.Accum() for _ in range(2 * len(cells))]
    if mine:
        res = run_grid([cells[i] for i in mine], B, detail=False)
        for i, r in zip(mine, res):
            local[2 * i], local[2 * i + 1] = r["accum"]
    merged = merge_ranked(gather_accums(local, group))
    return [(merged[2 * i], merged[2 * i + 1]) for i in range(len(cells))]


# ------------------------------------------------- HRS replicates and eps sweep (a19 / C5)
def gather_rows(local: np.ndarray, counts: List[int], group=None) -> np.ndarray:
    """All-gather every rank's [count_r, w] float64 rows -> the [sum(counts), w] array in rank
    order, identical on all ranks.  Shards differ in size by at most one row, so each rank pads
    to the largest (one all_gather of equal tensors; RCCL from device memory under 'nccl')."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    w = local.shape[1] if local.ndim == 2 else 6
    mx = max(counts) if counts else 0
    buf = np.zeros((mx, w), dtype=np.float64)
    buf[:counts[rank]] = local.reshape(counts[rank], w)
    t = torch.from_numpy(buf)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return np.concatenate([o.cpu().numpy()[:c] for o, c in zip(outs, counts)]) if counts else buf


def run_hrs_distributed(age_z, bmi_z, lam_age, lam_bmi, eps, reps, group=None, rep_begin=0, **kw):
    """The HRS replicates of one eps (real-data-sims.R:411-436; BASELINE C5's 1e6 replicates) over
    G ranks: rank g runs the contiguous replicate range shard(reps, g, G) with dcor.hrs.hrs_replicates
    (any rng / mode), and the records are all-gathered in rank order.  A replicate's numbers depend
    only on (seeds, replicate index) -- Philox counters, or the reference's per-run set.seed in
    rng='R' -- so the [reps, 6] result, identical on all ranks, equals one process's
    hrs_replicates(..., reps, rep_begin) byte for byte."""
    import torch.distributed as dist

    from .hrs import hrs_replicates
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    b0, nb = shard(reps, rank, world)
    local = (hrs_replicates(age_z, bmi_z, lam_age, lam_bmi, eps, nb, rep_begin=rep_begin + b0, **kw)
             if nb > 0 else np.zeros((0, 6)))
    return gather_rows(local, [shard(reps, r, world)[1] for r in range(world)], group)


def sweep_shard(n_eps: int, reps: int, rank: int, world: int):
    """Rank `rank`'s part of an eps sweep of n_eps x reps runs: the contiguous range of the flattened
    (eps index, run) space, as (eps index 0-based, first run, count) segments.  At the reference's
    23 x 200 runs each rank gets whole launches of several hundred runs instead of reps / G per eps."""
    b0, nb = shard(n_eps * reps, rank, world)
    segs, i = [], b0
    while i < b0 + nb:
        e, r = divmod(i, reps)
        c = min(reps - r, b0 + nb - i)
        segs.append((e, r, c))
        i += c
    return segs


def eps_sweep_distributed(age_z, bmi_z, lam_age, lam_bmi, eps_grid=None, reps=None, nsim=2000, rng="philox",
                          group=None):
    """dcor.hrs.eps_sweep (real-data-sims.R:345-448) over G ranks: the flattened (eps, run) space
    is split into contiguous per-rank ranges (sweep_shard); a rank runs its segments with the sweep's
    per-eps keys (Philox 10 + 1000 idx / 20 + 1000 idx: hrs.sweep_segments over HIP streams; rng='R':
    the reference's per-run set.seed, one hrs_replicates call per segment); the records are
    all-gathered in rank order and the per-eps summaries built from them on every rank.  Equal to the single-process eps_sweep: runs byte for byte, summaries
    identical."""
    import torch.distributed as dist

    from . import hrs
    eps_grid = hrs.EPS_GRID if eps_grid is None else eps_grid
    reps = hrs.R_PER_EPS if reps is None else reps
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    segs = sweep_shard(len(eps_grid), reps, rank, world)
    if rng == "philox" and segs:
        local = hrs.sweep_segments(age_z, bmi_z, lam_age, lam_bmi, eps_grid, segs, nsim=nsim)
    else:
        parts = [hrs.hrs_replicates(age_z, bmi_z, lam_age, lam_bmi, eps_grid[e], c, seed_ni=10 + 1000 * (e + 1),
                                    seed_int=20 + 1000 * (e + 1), nsim=nsim, rng=rng, eps_idx=e + 1, rep_begin=r0)
                 for e, r0, c in segs]
        local = np.concatenate(parts) if parts else np.zeros((0, 6))
    counts = [shard(len(eps_grid) * reps, r, world)[1] for r in range(world)]
    runs = gather_rows(local, counts, group).reshape(len(eps_grid), reps, 6)
    return hrs.sweep_summaries(eps_grid, runs)
