"""R-stream mode: the simulation drivers with R's OWN random streams.

`run_sim_one(..., seed)` in R starts from set.seed(seed) and draws, replicate after
replicate, in the order of SURVEY.md Appendix A (vert-cor.R:364,392-419;
ver-cor-subG.R:169,174-198).  This module runs the same cells on the GPU through
`dcor_rstream_grid_run`: one Mersenne-Twister wave per cell (R's generator, seeding,
inversion rnorm, exp_rand, rbinom, extraDistr rlaplace, mvrnorm's LAPACK eigen factor), then the
pre-materialised estimator kernels.  Replicate b of a cell is the reference's replicate b for
that seed, up to libm rounding of log ("R-stream mode").  The default engine
(`dcor.sim`) keeps the counter-based Philox streams, which shard over GPUs by replicate; this
mode shards by cell, like the reference's mclapply.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import lib
from .api import batch_geometry
from .sim import CellSpec, detail_frame, finalize

R_DGPS = ("gaussian", "bernoulli", "bounded_factor", "mix_gaussian")


def run_grid(cells, B: int, detail: bool = True) -> list:
    """All cells, B replicates each, R streams -> [{'summary', 'accum', 'detail'?}]."""
    cells = list(cells)
    nc = len(cells)
    arr = (_lib.Cell * nc)(*[c.to_c() for c in cells])
    acc = (_lib.Accum * (2 * nc))()
    det = (_lib.RepOut * (nc * B))() if detail else None
    _lib.check(lib.dcor_rstream_grid_run(arr, nc, B, acc, det))
    rec = np.ctypeslib.as_array(C.cast(det, C.POINTER(C.c_double)), shape=(nc * B * 6,)).reshape(
        nc, B, 6).copy() if detail else None
    out = []
    for i, c in enumerate(cells):
        ni, it = acc[2 * i], acc[2 * i + 1]
        res = {"summary": {"NI": finalize(ni, c.rho), "INT": finalize(it, c.rho)}, "accum": (ni, it)}
        if detail:
            res["detail"] = detail_frame(rec[i], c.rho)
            res["records"] = rec[i]
        out.append(res)
    return out


def run_cell(cell: CellSpec, B: int, detail: bool = True) -> dict:
    return run_grid([cell], B, detail)[0]


def draws(cell: CellSpec, reps: int) -> dict:
    """The explicit inputs of R-stream replicates 0 .. reps-1 (rep-major host arrays)."""
    c = cell.to_c()
    n, nsim = cell.n, cell.nsim
    k, _ = batch_geometry(n, cell.eps1, cell.eps2, cell.family)
    a = {"X": np.zeros((reps, n)), "Y": np.zeros((reps, n)), "lap_ni_sc": np.zeros((reps, 4)),
         "lap_int_sc": np.zeros((reps, 4)), "lap_ni_x": np.zeros((reps, k)),
         "lap_ni_y": np.zeros((reps, k)), "flips": np.zeros((reps, (n + 31) // 32), dtype=np.uint32),
         "lap_local": np.zeros((reps, n)), "lap_scalar": np.zeros(reps),
         "mix_z": np.zeros((reps, nsim)), "mix_l": np.zeros((reps, nsim))}
    d = _lib.RsDraws()
    for key, v in a.items():
        ptr_t = C.POINTER(C.c_uint32) if v.dtype == np.uint32 else C.POINTER(C.c_double)
        setattr(d, key, v.ctypes.data_as(ptr_t))
    _lib.check(lib.dcor_rstream_draws(C.byref(c), reps, C.byref(d)))
    return a


def words(seed: int, count: int) -> np.ndarray:
    """The first `count` tempered MT19937 words after set.seed(seed), from the GPU."""
    out = np.zeros(count, dtype=np.uint32)
    _lib.check(lib.dcor_rstream_words(int(seed), count, out.ctypes.data_as(C.POINTER(C.c_uint32))))
    return out
