"""Fused Monte-Carlo engine: grid cells, replicate drivers and summaries.

Replaces run_sim_one (vert-cor.R:356-444; ver-cor-subG.R:159-222) and the
expand.grid + mclapply grid drivers (vert-cor.R:486-597; ver-cor-subG.R:245-335).
Replicates run on the GPU (one workgroup each) from counter-based Philox streams
keyed by the cell seed, so a replicate's numbers depend only on (seed, rep) and
any split over launches or GPUs reproduces them bit for bit.
torch supplies device memory and the stream; all compute is in libdcor.so.
"""
from __future__ import annotations

import ctypes as C
import itertools
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib

DETAIL_COLS = ("ni_hat", "ni_low", "ni_up", "int_hat", "int_low", "int_up")


@dataclass
class CellSpec:
    """One (family, distribution, rho, eps, n) grid cell + run_sim_one arguments."""
    n: int
    rho: float
    eps1: float
    eps2: float
    family: str = "sign"            # "sign" (vert-cor.R) or "subG" (ver-cor-subG.R)
    dgp: str = "gaussian"           # "gaussian" | "bernoulli" | "bounded_factor" | "mix_gaussian"
    alpha: float = 0.05
    mu: Sequence[float] = (0.0, 0.0)
    sigma: Sequence[float] = (1.0, 1.0)
    eta1: float = 1.0
    eta2: float = 1.0
    normalise: bool = True
    ci_mode: str = "auto"
    nsim: int = 1000
    seed: int = 2025
    # gen_mix_gaussian arguments (ver-cor-subG.R:113-116 defaults)
    mix_mu0: Sequence[float] = (0.0, 0.0)
    mix_sigma0: Sequence[float] = (1.0, 1.0)
    mix_mu1: Sequence[float] = (3.0, 3.0)
    mix_sigma1: Sequence[float] = (2.0, 0.5)
    pi_mix: float = 0.5

    def to_c(self) -> _lib.Cell:
        c = _lib.Cell()
        c.family = _lib.FAMILY_SUBG if self.family == "subG" else _lib.FAMILY_SIGN
        c.dgp = {"gaussian": _lib.DGP_GAUSSIAN, "bernoulli": _lib.DGP_BERNOULLI,
                 "bounded_factor": _lib.DGP_BOUNDED_FACTOR,
                 "mix_gaussian": _lib.DGP_MIX_GAUSSIAN}[self.dgp]
        c.n = int(self.n)
        c.rho, c.eps1, c.eps2, c.alpha = float(self.rho), float(self.eps1), float(self.eps2), float(self.alpha)
        c.mu[0], c.mu[1] = float(self.mu[0]), float(self.mu[1])
        c.sigma[0], c.sigma[1] = float(self.sigma[0]), float(self.sigma[1])
        c.eta1, c.eta2 = float(self.eta1), float(self.eta2)
        c.normalise = int(bool(self.normalise))
        c.ci_mode = _lib.mode_code(self.ci_mode)
        c.nsim = int(self.nsim)
        c.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        for name, v in (("mix_mu0", self.mix_mu0), ("mix_sigma0", self.mix_sigma0),
                        ("mix_mu1", self.mix_mu1), ("mix_sigma1", self.mix_sigma1)):
            getattr(c, name)[0], getattr(c, name)[1] = float(v[0]), float(v[1])
        c.mix_pi = float(self.pi_mix)
        return c


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.DcorError(_lib.DCOR_ENODEV, "no GPU visible: the dcor engine has no CPU path")
    return torch


def _stream_ptr(stream) -> int:
    torch = _torch()
    s = torch.cuda.current_stream() if stream is None else stream
    return int(s.cuda_stream)


def simulate(cell: CellSpec, reps: int, rep_begin: int = 0, out=None, stream=None):
    """Replicates [rep_begin, rep_begin+reps) of `cell` -> float64 tensor [reps, 6] on the GPU
    (columns DETAIL_COLS).  Asynchronous on `stream` (default: torch's current stream)."""
    torch = _torch()
    if out is None:
        out = torch.empty((reps, 6), dtype=torch.float64, device="cuda")
    assert out.is_cuda and out.dtype == torch.float64 and out.is_contiguous() and out.shape[0] >= reps
    c = cell.to_c()
    check(lib.dcor_sim_launch(C.byref(c), int(rep_begin), int(reps), C.c_void_p(out.data_ptr()),
                              C.c_void_p(_stream_ptr(stream))))
    return out


def accumulate(records, rho: float, stream=None):
    """Deterministic per-method accumulators of device records -> (2, 20) int64/float view
    returned as a list of two _lib.Accum (host)."""
    torch = _torch()
    n = records.shape[0]
    acc = torch.empty(2 * C.sizeof(_lib.Accum), dtype=torch.uint8, device="cuda")
    check(lib.dcor_accumulate_launch(C.c_void_p(records.data_ptr()), int(n), float(rho),
                                     C.c_void_p(acc.data_ptr()), C.c_void_p(_stream_ptr(stream))))
    return acc


def accum_from_bytes(buf: bytes):
    a = (_lib.Accum * 2).from_buffer_copy(buf)
    return [a[0], a[1]]


def merge(accums):
    """Merge a rank-ordered list of Accum (double-double sums; deterministic)."""
    out = _lib.Accum()
    for a in accums:
        lib.dcor_accum_merge(C.byref(out), C.byref(a))
    return out


def finalize(acc: _lib.Accum, rho: float) -> dict:
    s = _lib.Summary()
    lib.dcor_accum_finalize(C.byref(acc), float(rho), C.byref(s))
    return {"mse": s.mse, "bias": s.bias, "var": s.var, "coverage": s.coverage, "ci_length": s.ci_length}


def r_cover(rho: float, lo, up) -> np.ndarray:
    """R's `rho >= lo && rho <= up` (vert-cor.R:405) / vectorised `&` (ver-cor-subG.R:203) with
    three-valued logic: FALSE if either comparison is FALSE, NA (NaN) if neither is FALSE and one
    is NA, else TRUE -- the rule the device accumulator applies (k_accumulate)."""
    lo = np.asarray(lo, dtype=np.float64)
    up = np.asarray(up, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        f1 = ~np.isnan(lo) & ~(rho >= lo)
        f2 = ~np.isnan(up) & ~(rho <= up)
    cov = np.where(np.isnan(lo) | np.isnan(up), np.nan, 1.0)
    cov[f1 | f2] = 0.0
    return cov


def detail_frame(rec: np.ndarray, rho: float) -> dict:
    """run_sim_one's `detail` (vert-cor.R:367-417; ver-cor-subG.R:170-206) from the six
    per-replicate numbers, columns in ver-cor-subG.R's order (tables.DETAIL_ORDER[:13])."""
    rec = np.asarray(rec, dtype=np.float64).reshape(-1, 6)
    d = {"repl": np.arange(1, rec.shape[0] + 1)}
    for i, name in enumerate(DETAIL_COLS):
        d[name] = rec[:, i]
    for m in ("ni", "int"):
        d[f"{m}_se2"] = (d[f"{m}_hat"] - rho) ** 2
    for m in ("ni", "int"):
        d[f"{m}_cover"] = r_cover(rho, d[f"{m}_low"], d[f"{m}_up"])
    for m in ("ni", "int"):
        d[f"{m}_ci_len"] = d[f"{m}_up"] - d[f"{m}_low"]
    return d


def run_cell(cell: CellSpec, B: int, detail: bool = True, chunk: int = 1 << 16, stream=None) -> dict:
    """All B replicates of one cell on the current GPU -> {'detail', 'summary'}.  With a
    `stream`, buffers are allocated, filled and copied back on that stream (torch's D2H copy
    runs on the current stream, so the loop runs with `stream` current)."""
    torch = _torch()
    recs = []
    accs = []
    s = torch.cuda.current_stream() if stream is None else stream
    with torch.cuda.stream(s):
        buf = torch.empty((min(B, chunk), 6), dtype=torch.float64, device="cuda")
        for r0 in range(0, B, chunk):
            nr = min(chunk, B - r0)
            simulate(cell, nr, r0, out=buf, stream=s)
            a = accumulate(buf[:nr], cell.rho, stream=s)
            accs.extend(accum_from_bytes(a.cpu().numpy().tobytes()))
            if detail:
                recs.append(buf[:nr].cpu().numpy().copy())
    ni = merge(accs[0::2])
    it = merge(accs[1::2])
    summary = {"NI": finalize(ni, cell.rho), "INT": finalize(it, cell.rho)}
    res = {"summary": summary, "accum": (ni, it)}
    if detail:
        res["detail"] = detail_frame(np.concatenate(recs), cell.rho)
    return res


# ---------------------------------------------------------- R-shaped drivers
def run_sim_one(n, rho, eps1, eps2, mu=(0.0, 0.0), sigma=(1.0, 1.0), B=1000, alpha=0.05,
                ci_mode="auto", normalise=True, seed=2025, dgp="gaussian", rng="philox") -> dict:
    """run_sim_one of vert-cor.R:356-444 (sign family; dgp='bernoulli' wires gen_bernoulli).
    rng='R' replays R's own stream for set.seed(seed) (dcor.rstream)."""
    cell = CellSpec(n=n, rho=rho, eps1=eps1, eps2=eps2, family="sign", dgp=dgp, alpha=alpha,
                    mu=mu, sigma=sigma, normalise=normalise, ci_mode=ci_mode, seed=seed)
    return _run(cell, B, rng)


def run_sim_one_subG(n, rho, eps1, eps2, dgp_fun="bounded_factor", dgp_args=None, B=1000,
                     alpha=0.05, use_subG=True, ci_mode="auto", seed=2025, rng="philox") -> dict:
    """run_sim_one of ver-cor-subG.R:159-222.  use_subG=FALSE routes to the sign family.
    rng='R' replays R's own stream for set.seed(seed) (dcor.rstream)."""
    args = dict(dgp_args or {})
    mix = {}
    if dgp_fun == "mix_gaussian":  # gen_mix_gaussian(mu0, sigma0, mu1, sigma1, pi_mix)
        mix = {k2: args[k1] for k1, k2 in (("mu0", "mix_mu0"), ("sigma0", "mix_sigma0"), ("mu1", "mix_mu1"),
                                           ("sigma1", "mix_sigma1"), ("pi_mix", "pi_mix")) if k1 in args}
    cell = CellSpec(n=n, rho=rho, eps1=eps1, eps2=eps2, family="subG" if use_subG else "sign",
                    dgp=dgp_fun, alpha=alpha, ci_mode=ci_mode, seed=seed,
                    mu=args.get("mu", (0.0, 0.0)), sigma=args.get("sigma", (1.0, 1.0)), **mix)
    return _run(cell, B, rng)


def _run(cell: CellSpec, B: int, rng: str) -> dict:
    if rng == "R":
        from .rstream import run_cell as run_cell_r
        return run_cell_r(cell, B)
    if rng != "philox":
        raise ValueError(f"rng must be 'philox' or 'R', not {rng!r}")
    return run_cell(cell, B)


# ------------------------------------------------------------------- grids
def expand_grid(n_grid, rho_grid, eps_pairs, **kw) -> list:
    """expand.grid(n, rho, eps_idx) with n fastest; seed = 1e6 + i (vert-cor.R:507-552)."""
    cells = []
    i = 0
    for e in eps_pairs:
        for rho in rho_grid:
            for n in n_grid:
                i += 1
                cells.append(CellSpec(n=n, rho=rho, eps1=e[0], eps2=e[1], seed=1_000_000 + i, **kw))
    return cells


def vert_cor_grid() -> list:
    """144-cell sign-family grid of vert-cor.R:486-499 (B = 250 there)."""
    return expand_grid([1000, 1500, 2500, 4000, 6000, 9000],
                       [0, 0.15, 0.3, 0.4, 0.5, 0.65, 0.8, 0.9],
                       [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5)],
                       family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0))


def subg_grid() -> list:
    """120-cell sub-G grid of ver-cor-subG.R:245-258 (bounded factor, B = 250)."""
    return expand_grid([2500, 4000, 6000, 9000, 12000],
                       [0, 0.15, 0.3, 0.4, 0.5, 0.65, 0.8, 0.9],
                       [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5)],
                       family="subG", dgp="bounded_factor")


def paper_grid(n_grid=(200, 400, 800, 1600, 3200)) -> list:
    """Legacy paper axes of vert-cor.R:19-40 crossed with both families (BASELINE C4)."""
    eps = [(0.2, 0.2), (0.5, 0.5), (1.0, 1.0), (1.5, 0.5), (0.5, 1.5)]
    rho = [0.0, 0.3, 0.8]
    out = []
    for fam, dgp, kw in (("sign", "gaussian", {}), ("sign", "bernoulli", {}),
                         ("subG", "gaussian", {}), ("subG", "bounded_factor", {})):
        out += expand_grid(list(n_grid), rho, eps, family=fam, dgp=dgp, **kw)
    return out


def headline_cell(n: int = 100_000) -> CellSpec:
    """BASELINE.json headline: sign family, mvrnorm mu=(.5,.5) sigma=(2,2), rho=.5, eps=(1,1)."""
    return CellSpec(n=n, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian",
                    mu=(0.5, 0.5), sigma=(2.0, 2.0), alpha=0.05, normalise=True, ci_mode="auto",
                    seed=1_000_073)


def _cells_array(cells):
    arr = (_lib.Cell * len(cells))()
    for i, c in enumerate(cells):
        arr[i] = c.to_c()
    return arr


def grid_launch(cells, rep_begin, rep_count, out=None, acc=None, stream=None):
    """The batched grid on the current GPU (dcor_grid_launch): replicates
    [rep_begin[i], rep_begin[i] + rep_count[i]) of every cell in a few launches.  Returns the
    device records (float64 [sum(rep_count), 6], cell-major) and the accumulators (uint8 tensor
    of 2 * len(cells) dcor_accum), asynchronous on `stream`."""
    torch = _torch()
    rb = np.ascontiguousarray(np.broadcast_to(np.asarray(rep_begin, dtype=np.int64), (len(cells),)))
    rc = np.ascontiguousarray(np.broadcast_to(np.asarray(rep_count, dtype=np.int64), (len(cells),)))
    tot = int(rc.sum())
    if out is None:
        out = torch.empty((max(tot, 1), 6), dtype=torch.float64, device="cuda")
    if acc is None:
        acc = torch.empty(2 * len(cells) * C.sizeof(_lib.Accum), dtype=torch.uint8, device="cuda")
    assert out.is_cuda and out.dtype == torch.float64 and out.is_contiguous() and out.shape[0] >= tot
    arr = _cells_array(cells)
    I64 = C.POINTER(C.c_int64)
    check(lib.dcor_grid_launch(arr, len(cells), rb.ctypes.data_as(I64), rc.ctypes.data_as(I64),
                               C.c_void_p(out.data_ptr()), C.c_void_p(acc.data_ptr()),
                               C.c_void_p(_stream_ptr(stream))))
    return out[:tot], acc


def accums_from_bytes(buf: bytes, ncells: int):
    a = (_lib.Accum * (2 * ncells)).from_buffer_copy(buf)
    return [(a[2 * i], a[2 * i + 1]) for i in range(ncells)]


def run_grid(cells, B: int, detail: bool = False, devices=None) -> list:
    """Every cell's B replicates through dcor_grid_run_multi: batched launches, replicate ranges
    sharded over `devices` (HIP ids; None: every visible GPU), accumulators merged in device
    order.  Replaces the expand.grid + mclapply blocks (vert-cor.R:486-554;
    ver-cor-subG.R:245-296).  -> [{'summary', 'accum'[, 'detail']}] per cell."""
    _torch()
    nc = len(cells)
    arr = _cells_array(cells)
    acc = (_lib.Accum * (2 * nc))()
    rec = np.zeros((nc * B, 6)) if detail else None
    devs = None if devices is None else (C.c_int * len(devices))(*devices)
    check(lib.dcor_grid_run_multi(arr, nc, int(B), devs, 0 if devices is None else len(devices), acc,
                                  None if rec is None else rec.ctypes.data_as(C.POINTER(_lib.RepOut))))
    out = []
    for i, c in enumerate(cells):
        ni, it = acc[2 * i], acc[2 * i + 1]
        r = {"summary": {"NI": finalize(ni, c.rho), "INT": finalize(it, c.rho)}, "accum": (ni, it)}
        if detail:
            r["records"] = rec[i * B:(i + 1) * B]
            r["detail"] = detail_frame(r["records"], c.rho)
        out.append(r)
    return out
