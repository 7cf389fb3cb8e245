"""HRS BMI-vs-Age real-data study (real-data-sims.R) on the engine: panel ingest, DP
standardisation, the calibrated lambdas, and the replicate sweep of BASELINE config C5.

The reference loads `hrs_long_panel.rds`, keeps wave 2 complete cases of (agey_e, bmi)
(real-data-sims.R:13, 38-41), standardises both columns with a DP mean / sd
(real-data-sims.R:73-106, 273-287) and runs the NI and INT estimators on the standardised
panel (real-data-sims.R:290-323), then sweeps eps over seq(.25, 2.5, .1) with R = 200
replicates each (real-data-sims.R:345-448).

Ingesting the HRS panel itself waits for a data-licensing decision by the
project owner, so the repository ships no HRS microdata, nothing computed from them, and no
reader for them.  `standin_panel(n, rho)` is a generic synthetic panel of the same kind
(whole-year ages, one-decimal BMIs): each column is centred on its clip interval
(real-data-sims.R:260-261) with sd = interval width / 4; n and rho are the caller's.
"""
from __future__ import annotations

import math

import numpy as np

# real-data-sims.R:260-270
AGE_LO, AGE_HI = 45.0, 90.0
BMI_LO, BMI_HI = 15.0, 35.0
EPS_MEAN, EPS_M2 = 0.10, 0.10
EPS_CORR = 2.0
# seq(0.25, 2.5, by = 0.1): R's seq.default computes from + (0:n) * by without rounding, so
# e.g. the 7th value is 0.8500000000000001 (R prints 0.85); which(eps_grid == eps) matches these.
EPS_GRID = tuple(0.25 + i * 0.1 for i in range(23))
R_PER_EPS = 200
NI_SEED, INT_SEED = 231, 322                                     # set.seed (:289, :312)


def standin_panel(n: int, rho: float, seed: int = 2):
    """Synthetic raw (age, bmi): whole-year ages and one-decimal BMIs from a bivariate normal
    centred on the clip intervals with sd = width / 4 and correlation rho."""
    g = np.random.default_rng(seed)
    za = g.standard_normal(n)
    zb = rho * za + math.sqrt(1.0 - rho * rho) * g.standard_normal(n)
    age = np.round(0.5 * (AGE_LO + AGE_HI) + 0.25 * (AGE_HI - AGE_LO) * za)
    bmi = np.round(0.5 * (BMI_LO + BMI_HI) + 0.25 * (BMI_HI - BMI_LO) * zb, 1)
    return age, bmi


def standardize_panel(age, bmi, lap=None, rng=None):
    """dp_sd of both columns, standardize_dp, lambda_from_priv (real-data-sims.R:273-287).
    lap: optional unit Laplace draws [age mean, age m2, bmi mean, bmi m2]."""
    from . import api
    lap = np.asarray(api.unit_laplace(4, rng) if lap is None else lap, dtype=np.float64)
    age_priv = api.dp_sd(age, AGE_LO, AGE_HI, EPS_MEAN, EPS_M2, lap=lap[:2])
    bmi_priv = api.dp_sd(bmi, BMI_LO, BMI_HI, EPS_MEAN, EPS_M2, lap=lap[2:])
    age_z = api.standardize_dp(age, age_priv, AGE_LO, AGE_HI)
    bmi_z = api.standardize_dp(bmi, bmi_priv, BMI_LO, BMI_HI)
    ok = ~(np.isnan(age_z) | np.isnan(bmi_z))                      # drop_na (:282)
    return {"age_z": np.ascontiguousarray(age_z[ok]), "bmi_z": np.ascontiguousarray(bmi_z[ok]),
            "age_priv": age_priv, "bmi_priv": bmi_priv,
            "lambda_age_z": api.lambda_from_priv(AGE_LO, AGE_HI, age_priv),
            "lambda_bmi_z": api.lambda_from_priv(BMI_LO, BMI_HI, bmi_priv)}


# ------------------------------------------------------------ replicate sweep (a19 / C5)
# On-device unit-noise streams of one HRS replicate (dcor_draws_launch / dcor_perm_launch
# sites).  The reference reseeds per run with set.seed(10 + 37 rep + 1000 idx) (NI) and
# set.seed(20 + 41 rep + 1000 idx) (INT) (real-data-sims.R:404, 423); here the per-eps seed
# is the Philox key and the replicate index is the counter, so replicates are independent
# streams and any split over launches or GPUs reproduces them exactly.
SITE_NI_LAP_X, SITE_NI_LAP_Y, SITE_INT_LOCAL, SITE_INT_CENTRAL, SITE_MIX_Z, SITE_MIX_L = 11, 12, 13, 14, 15, 16
DRAW_LAPLACE, DRAW_NORMAL = 0, 1


def r_seeds(idx: int, reps, rep_begin: int = 0):
    """The reference's per-run seeds at eps index idx (1-based, which(eps_grid == eps)) for
    runs rep = rep_begin+1 .. rep_begin+reps: set.seed(10 + 37 rep + 1000 idx) before
    run_NI_once and set.seed(20 + 41 rep + 1000 idx) before run_INT_once
    (real-data-sims.R:404, 423)."""
    rep = np.arange(rep_begin + 1, rep_begin + reps + 1, dtype=np.int64)
    return ((10 + 37 * rep + 1000 * idx).astype(np.int32), (20 + 41 * rep + 1000 * idx).astype(np.int32))


def _philox_draws(seed_ni, seed_int, rb, nr, n, k, m, nsim, bufs, sp):
    """The Philox unit-noise arrays of runs rb .. rb+nr-1 into bufs (perm, lap_x, lap_y,
    lap_local, lap_central, mix_z, mix_l), enqueued on stream sp."""
    import ctypes as C

    from . import _lib
    P = lambda t: C.c_void_p(t.data_ptr())
    perm, lx, ly, ll, lc, mz, ml = bufs
    chk = _lib.check
    chk(_lib.lib.dcor_perm_launch(seed_ni, _lib.SITE_PERM, rb, nr, n, k * m, P(perm), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_LAPLACE, seed_ni, SITE_NI_LAP_X, rb, nr, k, P(lx), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_LAPLACE, seed_ni, SITE_NI_LAP_Y, rb, nr, k, P(ly), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_LAPLACE, seed_int, SITE_INT_LOCAL, rb, nr, n, P(ll), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_LAPLACE, seed_int, SITE_INT_CENTRAL, rb, nr, 1, P(lc), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_NORMAL, seed_int, SITE_MIX_Z, rb, nr, nsim, P(mz), sp))
    chk(_lib.lib.dcor_draws_launch(DRAW_LAPLACE, seed_int, SITE_MIX_L, rb, nr, nsim, P(ml), sp))


def _premat_launch(X, Y, pn, n, nr, eps, lam_age, lam_bmi, lam_r, delta, nsim, alpha, bufs, out, sp):
    """One pre-materialised HRS launch over the panel pn: nr runs from the noise in bufs into
    out[:nr] (dcor_premat_subg_panel_launch), enqueued on stream sp."""
    import ctypes as C

    from . import _lib
    perm, lx, ly, ll, lc, mz, ml = bufs
    d = _lib.PrematSubg(n=n, reps=nr, eps1=eps, eps2=eps, eta1=1.0, eta2=1.0, alpha=alpha, hrs=1,
                        lam_x=lam_age, lam_y=lam_bmi, lam_s=lam_age, lam_o=lam_bmi, lam_r=lam_r,
                        delta=delta, nsim=nsim, X=X.data_ptr(), Y=Y.data_ptr(), xy_stride=0,
                        perm=perm.data_ptr(), lap_ni_x=lx.data_ptr(), lap_ni_y=ly.data_ptr(),
                        lap_local=ll.data_ptr(), lap_central=lc.data_ptr(), mix_z=mz.data_ptr(),
                        mix_l=ml.data_ptr())
    _lib.check(_lib.lib.dcor_premat_subg_panel_launch(C.byref(d), pn, C.c_void_p(out.data_ptr()), sp))


def hrs_replicates(age_z, bmi_z, lam_age, lam_bmi, eps, reps, seed_ni=NI_SEED, seed_int=INT_SEED,
                   nsim=2000, rep_begin=0, chunk=8192, alpha=0.05, keep_noise=False, rng="philox",
                   eps_idx=None, mode="premat"):
    """`reps` NI + INT replicates of the HRS estimators on one standardised panel at one eps:
    correlation_NI_subG(lambda_X = lam_age, lambda_Y = lam_bmi) and ci_INT_subG(AGE sends,
    lambda_receiver_from_noise, delta_clip = 1/n) (real-data-sims.R:357-400).  The panel is
    encoded once (dcor_panel_create); noise is generated in HBM per chunk and streamed by the
    pre-materialised kernel.  Returns float64 [reps, 6] (ni_hat, ni_lo, ni_hi, int_hat, int_lo,
    int_hi) and, with keep_noise, the host copies of every noise array.

    rng='R' replays the reference's own streams instead: run rep (1-based, rep_begin + 1 ..)
    draws its NI noise after set.seed(10 + 37 rep + 1000 eps_idx) and its INT noise after
    set.seed(20 + 41 rep + 1000 eps_idx) (dcor_rstream_hrs_draws), so every run is the
    reference's run for that seed; seed_ni / seed_int are then unused.

    mode='fused' (rng='philox' only) draws the same Philox noise inside the streaming kernel
    (dcor_hrs_fused_launch) instead of materialising it in HBM: the results equal the
    pre-materialised pipeline's to within its compensated sums' rounding.  Any panel: a
    dictionary-coded one (at most 256 distinct values per column) runs from LDS codes, a
    continuous one gathers its clipped values from L2 (n <= 65536) or is materialised per
    chunk (larger n)."""
    import ctypes as C

    import torch

    from . import _lib, api
    if rng not in ("philox", "R"):
        raise ValueError(f"rng must be 'philox' or 'R', not {rng!r}")
    if mode not in ("premat", "fused"):
        raise ValueError(f"mode must be 'premat' or 'fused', not {mode!r}")
    if mode == "fused" and (rng != "philox" or keep_noise):
        raise ValueError("mode='fused' draws Philox noise in the kernel: rng='philox', keep_noise=False")
    if rng == "R" and eps_idx is None:
        raise ValueError("rng='R' needs eps_idx (the 1-based position of eps in the sweep)")
    X = torch.as_tensor(np.ascontiguousarray(age_z, dtype=np.float64), device="cuda")
    Y = torch.as_tensor(np.ascontiguousarray(bmi_z, dtype=np.float64), device="cuda")
    n = int(X.shape[0])
    k, m = api.batch_geometry(n, eps, eps, "subG", hrs=True)
    delta = 1.0 / n
    lam_r = api.lambda_receiver_from_noise(lam_age, lam_bmi, eps, delta)
    P = lambda t: C.c_void_p(t.data_ptr())
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    pn = C.c_void_p()
    _lib.check(_lib.lib.dcor_panel_create(P(X), P(Y), n, sp, C.byref(pn)))
    cr = min(chunk, max(1, reps))
    f64 = dict(dtype=torch.float64, device="cuda")
    if mode == "fused":
        out = torch.empty((reps, 6), **f64)
        try:
            for r0 in range(0, reps, cr):
                nr = min(cr, reps - r0)
                d = _lib.PrematSubg(n=n, reps=nr, eps1=eps, eps2=eps, eta1=1.0, eta2=1.0, alpha=alpha,
                                    hrs=1, lam_x=lam_age, lam_y=lam_bmi, lam_s=lam_age, lam_o=lam_bmi,
                                    lam_r=lam_r, delta=delta, nsim=nsim, X=X.data_ptr(), Y=Y.data_ptr(),
                                    xy_stride=0)
                _lib.check(_lib.lib.dcor_hrs_fused_launch(C.byref(d), pn, seed_ni, seed_int,
                                                          rep_begin + r0, P(out[r0:]), sp))
            return out.cpu().numpy()
        finally:
            _lib.lib.dcor_panel_destroy(pn)
    if rng == "philox" and not keep_noise:
        # the launch chain natively (dcor_hrs_sweep_launch), one segment per chunk of cr runs
        out = torch.empty((max(reps, 1), 6), **f64)
        try:
            _native_segments(X, Y, pn, lam_age, lam_bmi, nsim, alpha,
                             [(eps, seed_ni, seed_int, rep_begin + r0, min(cr, reps - r0), r0)
                              for r0 in range(0, reps, cr)], out, stream)
            return out[:reps].cpu().numpy()
        finally:
            _lib.lib.dcor_panel_destroy(pn)
    perm = torch.empty((cr, k * m), dtype=torch.int32, device="cuda")
    lx, ly = torch.empty((cr, k), **f64), torch.empty((cr, k), **f64)
    ll, lc = torch.empty((cr, n), **f64), torch.empty((cr,), **f64)
    mz, ml = torch.empty((cr, nsim), **f64), torch.empty((cr, nsim), **f64)
    out = torch.empty((reps, 6), **f64)
    noise = {key: [] for key in ("perm", "lap_x", "lap_y", "lap_local", "lap_central", "mix_z", "mix_l")}
    try:
        for r0 in range(0, reps, cr):
            nr = min(cr, reps - r0)
            rb = rep_begin + r0
            chk = _lib.check
            if rng == "R":
                sn, si = r_seeds(eps_idx, nr, rb)
                I32 = C.POINTER(C.c_int32)
                chk(_lib.lib.dcor_rstream_hrs_draws(n, k, m, nsim, nr, sn.ctypes.data_as(I32),
                                                    si.ctypes.data_as(I32), P(perm), P(lx), P(ly),
                                                    P(ll), P(lc), P(mz), P(ml), sp))
            else:
                _philox_draws(seed_ni, seed_int, rb, nr, n, k, m, nsim, (perm, lx, ly, ll, lc, mz, ml), sp)
            _premat_launch(X, Y, pn, n, nr, eps, lam_age, lam_bmi, lam_r, delta, nsim, alpha,
                           (perm, lx, ly, ll, lc, mz, ml), out[r0:], sp)
            if keep_noise:
                for key, t in (("perm", perm), ("lap_x", lx), ("lap_y", ly), ("lap_local", ll),
                               ("lap_central", lc), ("mix_z", mz), ("mix_l", ml)):
                    noise[key].append(t[:nr].cpu().numpy().copy())
        res = out.cpu().numpy()
    finally:
        _lib.lib.dcor_panel_destroy(pn)
    if keep_noise:
        return res, {key: np.concatenate(v) for key, v in noise.items()}, {"k": k, "m": m, "lam_r": lam_r,
                                                                           "delta": delta}
    return res


def _summ(method, eps, hat, lo, hi) -> dict:
    """real-data-sims.R:408-418 / 427-437: means and type-7 quantiles (NA propagates)."""
    def q(v, p):
        return float("nan") if np.isnan(v).any() else float(np.quantile(v, p))
    return {"method": method, "eps_corr": eps, "rho_hat_mean": float(np.mean(hat)),
            "ci_low_mean": float(np.mean(lo)), "ci_high_mean": float(np.mean(hi)),
            "ci_low_q10": q(lo, 0.10), "ci_high_q90": q(hi, 0.90)}


def _native_segments(X, Y, pn, lam_age, lam_bmi, nsim, alpha, rowsegs, out, stream):
    """Enqueue (eps, seed_ni, seed_int, first run, count, output row) segments on `stream` with one
    dcor_hrs_sweep_launch: per segment the seven Philox noise arrays in one launch, then the
    pre-materialised panel kernels, records to out[row ..]."""
    import ctypes as C

    from . import _lib
    if not rowsegs:
        return
    n = int(X.shape[0])
    base = _lib.PrematSubg(n=n, reps=0, eps1=1.0, eps2=1.0, eta1=1.0, eta2=1.0, alpha=alpha, hrs=1,
                           lam_x=lam_age, lam_y=lam_bmi, lam_s=lam_age, lam_o=lam_bmi, lam_r=float("nan"),
                           delta=1.0 / n, nsim=nsim, X=X.data_ptr(), Y=Y.data_ptr(), xy_stride=0)
    arr = (_lib.HrsSegment * len(rowsegs))(*[
        _lib.HrsSegment(eps=e, seed_ni=sn, seed_int=si, rep_begin=r0, reps=c, out_row=row)
        for e, sn, si, r0, c, row in rowsegs])
    _lib.check(_lib.lib.dcor_hrs_sweep_launch(C.byref(base), pn, arr, len(rowsegs),
                                              C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)))


_SIDE = {}


def _side_streams(ns):
    """ns HIP streams of the current device, created once per process (stream creation and
    destruction cost more than a sweep's launches)."""
    import torch
    dev = torch.cuda.current_device()
    pool = _SIDE.setdefault(dev, [])
    while len(pool) < ns:
        pool.append(torch.cuda.Stream(device=dev))
    return pool[:ns]


def sweep_segments(age_z, bmi_z, lam_age, lam_bmi, eps_grid, segs, nsim=2000, alpha=0.05, streams=1):
    """Philox pre-materialised runs of several (eps index 0-based, first run, count) segments of
    an eps sweep on one shared panel -> [sum(count), 6] float64 in segment order.  Each segment's
    runs equal hrs_replicates(eps_grid[e], count, seed_ni=10 + 1000 idx, seed_int=20 + 1000 idx,
    rep_begin=first) byte for byte (idx = e + 1; the same draws and kernels), but the panel is
    uploaded and encoded once and the per-eps launch chains run from one native call
    (dcor_hrs_sweep_launch) instead of eight launches from Python per eps; with streams > 1 the
    segments are dealt round-robin over that many HIP streams, one native call each.  The host
    waits once, at the end."""
    import ctypes as C

    import torch

    from . import _lib
    X = torch.as_tensor(np.ascontiguousarray(age_z, dtype=np.float64), device="cuda")
    Y = torch.as_tensor(np.ascontiguousarray(bmi_z, dtype=np.float64), device="cuda")
    n = int(X.shape[0])
    rows = np.cumsum([0] + [c for _, _, c in segs])
    total = int(rows[-1])
    main = torch.cuda.current_stream()
    pn = C.c_void_p()
    _lib.check(_lib.lib.dcor_panel_create(C.c_void_p(X.data_ptr()), C.c_void_p(Y.data_ptr()), n,
                                          C.c_void_p(main.cuda_stream), C.byref(pn)))
    out = torch.empty((max(total, 1), 6), dtype=torch.float64, device="cuda")
    rowsegs = [(eps_grid[e], 10 + 1000 * (e + 1), 20 + 1000 * (e + 1), r0, c, int(rows[j]))
               for j, (e, r0, c) in enumerate(segs)]
    ns = max(1, min(streams, len(segs)))
    side = _side_streams(ns) if ns > 1 else [main]
    try:
        for j, s in enumerate(side):
            if s is not main:
                s.wait_stream(main)              # X, Y, the panel and out exist before any launch
            _native_segments(X, Y, pn, lam_age, lam_bmi, nsim, alpha, rowsegs[j::ns], out, s)
        for s in side:
            if s is not main:
                main.wait_stream(s)
        res = out[:total].cpu().numpy()
    finally:
        for s in side:
            s.synchronize()
        _lib.lib.dcor_panel_destroy(pn)
    return res


def eps_sweep(age_z, bmi_z, lam_age, lam_bmi, eps_grid=EPS_GRID, reps=R_PER_EPS, nsim=2000,
              rng="philox", streams=1):
    """The replicate sweep of real-data-sims.R:345-448: for every eps in seq(.25, 2.5, .1),
    `reps` NI and INT runs (Philox keys 10 + 1000 idx and 20 + 1000 idx, idx 1-based as
    which(eps_grid == eps); rng='R': the reference's own per-run set.seed streams) and the
    per-eps summaries ni_mean / int_mean.  rng='philox' runs every eps on one encoded panel from
    one native call per HIP stream (sweep_segments); the runs equal one hrs_replicates call per eps."""
    if rng == "philox":
        segs = [(e, 0, reps) for e in range(len(eps_grid))]
        runs = sweep_segments(age_z, bmi_z, lam_age, lam_bmi, eps_grid, segs, nsim=nsim, streams=streams)
        return sweep_summaries(eps_grid, runs.reshape(len(eps_grid), reps, 6))
    runs = [hrs_replicates(age_z, bmi_z, lam_age, lam_bmi, eps, reps, seed_ni=10 + 1000 * idx,
                           seed_int=20 + 1000 * idx, nsim=nsim, rng=rng, eps_idx=idx)
            for idx, eps in enumerate(eps_grid, start=1)]
    return sweep_summaries(eps_grid, np.stack(runs))


def sweep_summaries(eps_grid, runs) -> dict:
    """The sweep's per-eps summaries from its runs [n_eps, reps, 6] (real-data-sims.R:408-437);
    dcor.dist.eps_sweep_distributed builds the same from the ranks' gathered runs.  Vectorised over
    eps; every value equals _summ's per-eps one (same reductions along contiguous rows)."""
    runs = np.asarray(runs, dtype=np.float64)
    cols = [np.ascontiguousarray(runs[:, :, j]) for j in range(6)]     # [n_eps, reps] each
    mean = [c.mean(axis=1) for c in cols]

    def q(c, p):                                                       # type 7; a NaN row -> NaN
        v = np.quantile(c, p, axis=1) if c.shape[1] else np.full(c.shape[0], np.nan)
        return np.where(np.isnan(c).any(axis=1), np.nan, v)
    lo_q = {1: q(cols[1], 0.10), 4: q(cols[4], 0.10)}
    hi_q = {2: q(cols[2], 0.90), 5: q(cols[5], 0.90)}

    def summ(method, j, i, eps):
        return {"method": method, "eps_corr": eps, "rho_hat_mean": float(mean[j][i]),
                "ci_low_mean": float(mean[j + 1][i]), "ci_high_mean": float(mean[j + 2][i]),
                "ci_low_q10": float(lo_q[j + 1][i]), "ci_high_q90": float(hi_q[j + 2][i])}
    ni_mean = [summ("NI", 0, i, eps) for i, eps in enumerate(eps_grid)]
    int_mean = [summ("INT", 3, i, eps) for i, eps in enumerate(eps_grid)]
    return {"eps": list(eps_grid), "runs": runs, "ni_mean": ni_mean, "int_mean": int_mean}
