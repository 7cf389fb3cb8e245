"""bench_configs.py -- the BASELINE.json configs beyond the headline (one JSON line each).

C1  vert-cor.R sign family n=1000 rho=.5 eps=(1,1), 1000 reps: GPU vs CPU oracle (1 and nproc-1 threads)
C2  Bernoulli sign-family grid n=1e4, 8 rho x 3 eps, 1e4 reps/cell (fused kernels)
C3  Gaussian + mixquant grid n=1e6, 8 rho x 3 eps, 1e5 reps/cell (the config's size; --c3-reps)
C4  legacy paper sweep: {sign: gaussian, bernoulli; sub-G: gaussian, bounded factor} x rho {0,.3,.8}
    x 5 eps pairs x n {200..3200, 1e4, 1e5, 1e6}, B=1000 (vert-cor.R:40) and 1e5 at n=1e6
C5  HRS BMI-vs-Age pre-materialised streaming (synthetic stand-in panel n=19,433, eps=2): noise
    generated on device into HBM, then the streaming kernel is timed -> replicates/s and HBM GB/s
S   sub-G fused, bounded factor, n=1e5, rho=.5, eps=(1,1)
VG  vert-cor.R's own 144-cell sign grid (vert-cor.R:486-499) at its B = 250, Philox mode, batched
    launches (dcor_grid_run_multi) vs the per-cell launch loop
SG  ver-cor-subG.R's own 120-cell sub-G grid (ver-cor-subG.R:245-258) at B = 250, likewise
R1  R-stream mode (R's own Mersenne-Twister streams) on the C1 cell: GPU vs the
    CPU restatement (1 thread)
RG  R-stream mode on vert-cor.R's own 144-cell sign-family grid, B = 250 (vert-cor.R:486-553)
RH  R-stream HRS sweep: real-data-sims.R's 23 eps x 200 runs with its own per-run set.seed
    streams (4,600 NI + 4,600 INT runs) on a stand-in panel n = 19,433
Run on one GPU: python bench_configs.py [--only C2,C5] > profiles/rNN_configs.jsonl
Multi-GPU (C3, C4: the configs BASELINE names for 8 GPUs): python bench_configs.py --gpus N --only C3,C4
starts N rank processes (one per GPU, torch.distributed over RCCL; or runs under torchrun), each
running its contiguous replicate shard of every cell (dcor.dist.run_grid_distributed), the
per-cell accumulators all-gathered once; total work is fixed (strong scaling) and the time is the
max over ranks.  --dry-run forms the group over gloo on the CPU and prints the shard plan.
"""
import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-correlation_amd"))
sys.path.insert(0, ROOT)

W_SAMPLE = {"gaussian": 260, "bernoulli": 120, "bounded_factor": 292}
FP64_PEAK_UNITS = 3.93e13
HBM_PEAK = 8.0e12


def timed(fn, reps=3, inner=1):
    """Best of `reps` timings of `inner` back-to-back calls (per call)."""
    import torch
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(inner):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / inner)
    return best


def grid_units(cells, B):
    from dcor.api import batch_geometry
    tot = 0.0
    for c in cells:
        try:
            k, m = batch_geometry(c.n, c.eps1, c.eps2, "subG" if c.family == "subG" else "sign")
        except Exception:
            k = 0
        tot += B * (W_SAMPLE[c.dgp] * c.n + 183 * k + 2.0e5)
    return tot


def run_grid_batched(cells, B):
    """The grid through dcor_grid_run_multi on GPU 0: batched launches, accumulators to the host."""
    from dcor.sim import run_grid
    return run_grid(cells, B, devices=[0])


def run_grid_gpu(cells, B, chunk=1 << 15):
    """The per-cell launch loop (dcor_sim_launch + dcor_accumulate_launch per cell): the A/B
    reference for the batched grid."""
    import torch
    from dcor.sim import simulate, accumulate
    buf = torch.empty((min(B, chunk), 6), dtype=torch.float64, device="cuda")
    acc = []
    for c in cells:
        for r0 in range(0, B, chunk):
            nr = min(chunk, B - r0)
            simulate(c, nr, r0, out=buf)
            acc.append(accumulate(buf[:nr], c.rho))
    return acc


# config line -> its committed rocprofv3 summary (per-kernel times and counters)
PROFILE_OF = {"VG": "vg", "SG": "sg", "C2": "c2", "C3": "c3", "C4": "c4", "S": "s", "C5": "c5",
              "C5-continuous": "c5c", "C5-fused": "c5f"}
# lines whose profile also holds a comparison run (VG, SG: the per-cell launch loop beside the
# timed batched grid call): only the timed path's kernels enter `physical`
TIMED_KERNELS = {"VG": ("k_grid_", "k_accumulate_pass", "k_accumulate_merge"),
                 "SG": ("k_grid_", "k_accumulate_pass", "k_accumulate_merge")}


def measured(name):
    """Where the line's per-kernel counters are (scripts/summarize_prof.py), whether that profile
    was taken on this tree's sources, and the physical fraction of each kernel that holds >= 5 % of
    the profiled GPU time: VALU time (the mix priced at measured absolute issue costs) over the
    SIMDs' cycles -- hardware-anchored, unlike the pinned convention `roofline_frac`, which prices
    the reference's work units and exceeds 1 when the kernels issue fewer instructions."""
    from bench import _profile, profile_stamp
    if name not in PROFILE_OF:
        return {}
    path = _profile(PROFILE_OF[name])
    if path is None:
        return {}
    head, fresh = profile_stamp(path)
    out = {"profile": os.path.relpath(path, ROOT), "profile_head": head, "profile_fresh": fresh}
    try:
        ks = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return out
    phys = {}
    for k, v in sorted(ks.items(), key=lambda kv: -kv[1].get("pct_time", 0.0)):
        if v.get("pct_time", 0.0) < 5.0:
            continue
        if name in TIMED_KERNELS and not k.replace("dcor::", "").startswith(TIMED_KERNELS[name]):
            continue
        phys[k.replace("dcor::", "")] = {
            "pct_time": v.get("pct_time"),
            "valu_time_frac": None if v.get("valu_time_frac") is None else round(v["valu_time_frac"], 4),
            "wait_any_frac": None if v.get("wait_any_frac") is None else round(v["wait_any_frac"], 4),
            "simd_cycles_per_valu_inst": None if v.get("cycles_per_valu_inst") is None
            else round(v["cycles_per_valu_inst"], 3),
            "hbm_bytes_per_dispatch": None if v.get("hbm_read_bytes_corrected") is None
            else v["hbm_read_bytes_corrected"] + (v.get("hbm_write_bytes") or 0.0)}
    out["physical"] = phys
    if name in TIMED_KERNELS:
        out["physical_kernels"] = "the timed batched grid call's kernels (%s*); pct_time is of the whole " \
            "profile, which also runs the per-cell comparison loop" % "*, ".join(TIMED_KERNELS[name])
    return out


def line(name, **kw):
    kw["config"] = name
    kw.update(measured(name))
    print(json.dumps(kw), flush=True)


def c1():
    from dcor.sim import CellSpec, simulate
    from oracle.oracle import sim_reps
    cell = CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    B = 1000
    t = timed(lambda: simulate(cell, B), reps=5, inner=20)
    t0 = time.perf_counter()
    sim_reps(cell.to_c(), 0, B, threads=1)
    t1 = time.perf_counter() - t0
    nthr = max(1, min(os.cpu_count() or 1, 16) - 1)
    t0 = time.perf_counter()
    sim_reps(cell.to_c(), 0, B, threads=nthr)
    tn = time.perf_counter() - t0
    line("C1", reps=B, gpu_s=t, gpu_reps_per_s=B / t, cpu_1thread_s=t1, cpu_1thread_reps_per_s=B / t1,
         cpu_threads=nthr, cpu_nthread_s=tn, cpu_nthread_reps_per_s=B / tn,
         note="CPU = oracle fused restatement (C); R's interpreted loop would be slower")


def c2():
    from dcor.sim import expand_grid
    cells = expand_grid([10_000], [0, 0.15, 0.3, 0.4, 0.5, 0.65, 0.8, 0.9],
                        [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5)], family="sign", dgp="bernoulli")
    B = 10_000
    t = timed(grid_call(cells, B), reps=2)
    u = grid_units(cells, B)
    line("C2", cells=len(cells), reps_per_cell=B, seconds=t, reps_per_s=len(cells) * B / t,
         roofline_frac=u / t / FP64_PEAK_UNITS)


C3_EPS = [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5)]


def c3_cells(eps=None):
    from dcor.sim import expand_grid
    return expand_grid([1_000_000], [0, 0.15, 0.3, 0.4, 0.5, 0.65, 0.8, 0.9],
                       eps or C3_EPS, family="sign", dgp="gaussian",
                       mu=(0.5, 0.5), sigma=(2.0, 2.0))


def c3(reps, eps=None):
    """eps: a subset of the config's eps pairs (per-batch-size measurement: m = 32, 8, 11)."""
    cells = c3_cells(eps)
    t = timed(grid_call(cells, reps), reps=1)
    u = grid_units(cells, reps)
    line("C3", cells=len(cells), reps_per_cell=reps, eps_pairs=eps or C3_EPS, seconds=t, reps_per_s=len(cells) * reps / t,
         roofline_frac=u / t / FP64_PEAK_UNITS,
         note="one dcor_grid_run_multi call on one GPU over every cell's reps_per_cell replicates, measured")


def c4_cells():
    """(every runnable cell, the n < 1e6 cells, the n = 1e6 cells, cells skipped for k < 1)."""
    from dcor.sim import paper_grid
    cells = paper_grid(n_grid=(200, 400, 800, 1600, 3200, 10_000, 100_000, 1_000_000))
    ok = []
    for c in cells:  # sign family needs k >= 1 (vert-cor.R:209): skip (n, eps) pairs where it fails
        m = math.ceil(8 / (c.eps1 * c.eps2))
        if c.family == "sign" and c.n // m < 1:
            continue
        ok.append(c)
    return ok, [c for c in ok if c.n < 1_000_000], [c for c in ok if c.n >= 1_000_000], len(cells) - len(ok)


def c4(B, B_big):
    """The paper sweep at its stated sizes: B replicates per cell (vert-cor.R:40), B_big for the
    n = 1e6 cells: two grid calls (one per B), timed together."""
    ok, small, big, nskip = c4_cells()
    g_small, g_big = grid_call(small, B), grid_call(big, B_big)

    def both():
        g_small()
        g_big()
    t = timed(both, reps=1)
    ts = timed(g_small, reps=1)
    tl = timed(lambda: run_grid_gpu(small, B), reps=1)
    reps = len(small) * B + len(big) * B_big
    u = grid_units(small, B) + grid_units(big, B_big)
    line("C4", cells=len(ok), cells_skipped_k_lt_1=nskip, reps_per_cell=B,
         reps_per_cell_n1e6=B_big, cells_n1e6=len(big), replicates=reps, seconds=t, reps_per_s=reps / t,
         roofline_frac=u / t / FP64_PEAK_UNITS, small_cells_seconds=ts,
         small_cells_per_cell_loop_seconds=tl, small_cells_per_cell_loop_reps_per_s=len(small) * B / tl,
         note="measured at the stated sizes: one dcor_grid_run_multi call for the n < 1e6 cells at B, one for "
              "the n = 1e6 cells at B_big; the per-cell launch loop (A/B reference) on the n < 1e6 cells")


def grid_call(cells, B):
    """One dcor_grid_run_multi call on GPU 0 with the cell table and the accumulator array built
    beforehand: the engine's cost for a whole grid (planning, table upload, the launches, the
    accumulators copied to the host) -- what R's dcor_grid pays per call -- without the Python
    post-processing of dcor.sim.run_grid."""
    from dcor import _lib
    from dcor.sim import _cells_array
    arr = _cells_array(cells)
    acc = (_lib.Accum * (2 * len(cells)))()
    dev = (_lib.C.c_int * 1)(0)
    return lambda: _lib.check(_lib.lib.dcor_grid_run_multi(arr, len(cells), int(B), dev, 1, acc, None))


def ref_grid(name, cells, B=250):
    """A reference grid at its own B: batched (one dcor_grid_run_multi call, accumulators on the
    host) vs the per-cell launch loop."""
    t = timed(grid_call(cells, B), reps=5, inner=4)
    tl = timed(lambda: run_grid_gpu(cells, B), reps=3)
    u = grid_units(cells, B)
    line(name, cells=len(cells), reps_per_cell=B, seconds=t, reps_per_s=len(cells) * B / t,
         roofline_frac=u / t / FP64_PEAK_UNITS, per_cell_loop_seconds=tl,
         per_cell_loop_reps_per_s=len(cells) * B / tl, speedup_vs_per_cell_loop=tl / t,
         note="Philox mode; seconds = one dcor_grid_run_multi call (planning, table upload, launches, the "
              "host copy of every cell's accumulators), best of 5 x 4 back-to-back calls")


def c5(R, panel="coded", rep_begin=0, emit=True):
    """panel 'coded': generic stand-in of the HRS kind (whole-year ages, one-decimal BMIs,
    dcor.hrs.standin_panel, DP-standardised as real-data-sims.R:273-287): the dictionary-coded
    LDS kernel.  panel 'continuous': every value distinct: the L2-gather kernel."""
    import numpy as np
    import torch
    from dcor import _lib
    n, eps = 19433, 2.0
    k, m = 9716, 2
    nsim = 2000
    g = np.random.default_rng(2)
    lam = (2.22, 2.60)
    if panel == "coded":
        from dcor import hrs
        age_raw, bmi_raw = hrs.standin_panel(n, -0.3)
        z = hrs.standardize_panel(age_raw, bmi_raw, lap=np.zeros(4))
        age, bmi = z["age_z"], z["bmi_z"]
        lam = (z["lambda_age_z"], z["lambda_bmi_z"])
    else:
        age = np.clip(g.normal(0.0, 1.0, n), -2.22, 2.22)     # synthetic stand-in (HRS not shipped)
        bmi = -0.19 * age + math.sqrt(1 - 0.19 ** 2) * g.normal(0.0, 1.0, n)
    X = torch.as_tensor(age, device="cuda")
    Y = torch.as_tensor(bmi, device="cuda")
    perm = torch.empty((R, k * m), dtype=torch.int32, device="cuda")
    lx = torch.empty((R, k), dtype=torch.float64, device="cuda")
    ly = torch.empty((R, k), dtype=torch.float64, device="cuda")
    ll = torch.empty((R, n), dtype=torch.float64, device="cuda")
    lc = torch.empty((R,), dtype=torch.float64, device="cuda")
    mz = torch.empty((R, nsim), dtype=torch.float64, device="cuda")
    ml = torch.empty((R, nsim), dtype=torch.float64, device="cuda")
    seed = 231
    P = lambda t: C.c_void_p(t.data_ptr())
    rb = rep_begin
    _lib.check(_lib.lib.dcor_perm_launch(seed, _lib.SITE_PERM, rb, R, n, k * m, P(perm), None))
    _lib.check(_lib.lib.dcor_draws_launch(0, seed, 11, rb, R, k, P(lx), None))
    _lib.check(_lib.lib.dcor_draws_launch(0, seed, 12, rb, R, k, P(ly), None))
    _lib.check(_lib.lib.dcor_draws_launch(0, seed, 13, rb, R, n, P(ll), None))
    _lib.check(_lib.lib.dcor_draws_launch(0, seed, 14, 0, 1, R, P(lc), None))
    _lib.check(_lib.lib.dcor_draws_launch(1, seed, 15, rb, R, nsim, P(mz), None))
    _lib.check(_lib.lib.dcor_draws_launch(0, seed, 16, rb, R, nsim, P(ml), None))
    out = torch.empty((R, 6), dtype=torch.float64, device="cuda")
    d = _lib.PrematSubg(n=n, reps=R, eps1=eps, eps2=eps, eta1=1.0, eta2=1.0, alpha=0.05, hrs=1,
                        lam_x=lam[0], lam_y=lam[1], lam_s=lam[0], lam_o=lam[1], lam_r=math.nan,
                        delta=math.nan, nsim=nsim, X=X.data_ptr(), Y=Y.data_ptr(), xy_stride=0,
                        perm=perm.data_ptr(), lap_ni_x=lx.data_ptr(), lap_ni_y=ly.data_ptr(),
                        lap_local=ll.data_ptr(), lap_central=lc.data_ptr(), mix_z=mz.data_ptr(),
                        mix_l=ml.data_ptr())
    pn = C.c_void_p()      # the panel is encoded once for the whole sweep (dcor_panel_create)
    _lib.check(_lib.lib.dcor_panel_create(P(X), P(Y), n, None, C.byref(pn)))
    t = timed(lambda: _lib.check(_lib.lib.dcor_premat_subg_panel_launch(C.byref(d), pn, P(out), None)),
              reps=5, inner=8)
    per_rep = 8 * n + 4 * k * m + 16 * k + 8 * nsim    # SURVEY §8d pinned: 404,648 B
    read_rep = 8 * n + 4 * k * m + 16 * k + 8 + 16 * nsim  # bytes the ABI actually reads (z, l apart)
    if not emit:
        _lib.check(_lib.lib.dcor_panel_destroy(pn))
        return t, per_rep
    cpu = c5_cpu(age, bmi, lam, eps, nsim, perm, lx, ly, ll, lc, mz, ml) if panel == "coded" else {}
    ok = C.c_int(-1)
    _lib.check(_lib.lib.dcor_panel_coded(pn, C.byref(ok)))
    _lib.check(_lib.lib.dcor_panel_destroy(pn))
    line("C5" if panel == "coded" else "C5-continuous", reps=R, seconds=t, reps_per_s=R / t,
         algorithmic_bytes_per_rep=per_rep, input_bytes_per_rep=read_rep,
         hbm_gbps=per_rep * R / t / 1e9, hbm_frac=per_rep * R / t / HBM_PEAK,
         input_gbps=read_rep * R / t / 1e9, panel=panel, **cpu,
         kernel=("dictionary-coded LDS panel (k_premat_subg_dict)" if ok.value else
                 "uncoded panel: INT stream (k_premat_subg_int) + NI LDS tiles (k_premat_subg_tiled) for m = 2, else L2 gathers"),
         note="synthetic stand-in panel; noise pre-generated on device (dcor_draws_launch / "
              "dcor_perm_launch); timed = one dcor_premat_subg_panel_launch (stream + epilogue) over a panel "
              "encoded once by dcor_panel_create")


def c5_cpu(age, bmi, lam, eps, nsim, perm, lx, ly, ll, lc, mz, ml, seconds=3.0):
    """CPU baseline for C5: the HRS NI + INT estimators (real-data-sims.R:115-147, 176-252)
    restated in C (oracle/dcor_oracle.c, R semantics), 1 thread, on the same panel and the
    first replicates' noise copied to the host; about `seconds` of work."""
    from oracle import oracle as orc
    host = [t[:64].cpu().numpy() for t in (perm, lx, ly, ll, lc, mz, ml)]
    done, t0 = 0, time.perf_counter()
    while done < 2000 and (done < 2 or time.perf_counter() - t0 < seconds):
        r = done % host[0].shape[0]  # the first (up to) 64 replicates' noise, cycled
        orc.ni_subg(age, bmi, eps, eps, hrs=1, lam_x=lam[0], lam_y=lam[1], perm=host[0][r],
                    lap_x=host[1][r], lap_y=host[2][r])
        orc.int_subg(age, bmi, eps, eps, hrs=1, lam_s=lam[0], lam_o=lam[1], lap_local=host[3][r],
                     lap_central=float(host[4][r]), mix_z=host[5][r], mix_l=host[6][r])
        done += 1
    el = time.perf_counter() - t0
    return {"cpu_1thread_reps_per_s": done / el,
            "cpu_sample": f"{done} NI + INT replicates of the HRS estimators on the same panel and noise "
                          f"(the first {host[0].shape[0]} replicates' noise, cycled) "
                          f"in {el:.2f} s: oracle/dcor_oracle.c (R semantics), 1 thread"}


def c5_e2e(R):
    """BASELINE C5 end to end: R NI + INT replicates of the HRS estimators at eps = 2 on a
    coded stand-in panel, noise generated on device per 8192-replicate chunk and streamed
    (dcor.hrs.hrs_replicates), results copied to the host."""
    import numpy as np
    import torch
    from dcor import hrs
    age_raw, bmi_raw = hrs.standin_panel(19433, -0.3)
    z = hrs.standardize_panel(age_raw, bmi_raw, lap=np.zeros(4))
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0)
    hrs.hrs_replicates(*args, 8192)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = hrs.hrs_replicates(*args, R, chunk=8192)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    line("C5-e2e", reps=R, seconds=t, reps_per_s=R / t, finite=bool(np.isfinite(res).all()),
         note="includes on-device Philox noise + keyed permutation generation per chunk and the "
              "D2H copy of all replicate records")


def c5_fused(R, panel="coded"):
    """C5 with the noise drawn inside the streaming kernel (dcor_hrs_fused_launch): the same
    Philox streams as C5-e2e, no HBM noise arrays; R NI + INT replicates, results to host.
    panel 'continuous': every value distinct (as c5's), the uncoded kernel k_hrs_fused_l2."""
    import numpy as np
    import torch
    from dcor import hrs
    if panel == "coded":
        age_raw, bmi_raw = hrs.standin_panel(19433, -0.3)
        z = hrs.standardize_panel(age_raw, bmi_raw, lap=np.zeros(4))
        args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0)
    else:
        g = np.random.default_rng(2)
        age = np.clip(g.normal(0.0, 1.0, 19433), -2.22, 2.22)
        bmi = -0.19 * age + math.sqrt(1 - 0.19 ** 2) * g.normal(0.0, 1.0, 19433)
        args = (age, bmi, 2.22, 2.60, 2.0)
    hrs.hrs_replicates(*args, 8192, mode="fused")  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = hrs.hrs_replicates(*args, R, chunk=65536, mode="fused")
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    line("C5-fused" if panel == "coded" else "C5-fused-continuous", reps=R, seconds=t, reps_per_s=R / t,
         finite=bool(np.isfinite(res).all()), panel=panel,
         kernel="k_hrs_fused (LDS codes)" if panel == "coded" else "k_hrs_fused_l2 (clipped panel in L2)",
         note="HRS replicates with in-kernel Philox noise (+ epilogue), the D2H copy of all replicate "
              "records included")


def hrs_sweep(R):
    """a19: the HRS eps sweep of real-data-sims.R:345-448 (23 eps x R runs, Philox per-eps keys,
    premat pipeline, one native launch chain) on one GPU, summaries built on the host."""
    import numpy as np
    import torch
    from dcor import hrs
    args = hrs_panel("coded")
    hrs.eps_sweep(*args, reps=R)    # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = hrs.eps_sweep(*args, reps=R)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    total = len(hrs.EPS_GRID) * R
    line("HS", replicates=total, seconds=t, reps_per_s=total / t, finite=bool(np.isfinite(res["runs"]).all()),
         note="23 eps x R NI + INT runs on the coded stand-in panel, encoded once, the eps' launch chains "
              "from one native call (hrs.sweep_segments), summaries (means, type-7 quantiles) on the host")


def subg():
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=100_000, rho=0.5, eps1=1.0, eps2=1.0, family="subG", dgp="bounded_factor", seed=5)
    R = 4096
    t = timed(lambda: simulate(cell, R), reps=3, inner=4)
    u = R * (292 * cell.n + 183 * 12500 + 2e5)
    line("S", reps=R, seconds=t, reps_per_s=R / t, roofline_frac=u / t / FP64_PEAK_UNITS)


def rstream_c1():
    from dcor import rstream
    from dcor.sim import CellSpec
    from oracle.oracle import rs_sim
    cell = CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    B = 1000
    t = timed(lambda: rstream.run_cell(cell, B, detail=False), reps=3)
    Bc = 200
    t0 = time.perf_counter()
    rs_sim(cell.to_c(), Bc)
    tc = (time.perf_counter() - t0) / Bc * B
    line("R1", reps=B, gpu_s=t, gpu_reps_per_s=B / t, cpu_1thread_s=tc, cpu_1thread_reps_per_s=B / tc,
         cpu_sample=f"{Bc} replicates timed, scaled to {B}",
         note="both sides replay R's stream for set.seed(1000073); GPU time includes allocation and D2H")


def rstream_grid():
    from dcor import rstream
    from dcor.sim import vert_cor_grid
    from oracle.oracle import rs_sim
    cells = vert_cor_grid()
    B = 250
    t = timed(lambda: rstream.run_grid(cells, B, detail=False), reps=1)
    # CPU restatement on a sample: the smallest and the largest n of the grid, 10 reps each
    samp = [cells[0], cells[5]]
    tc = 0.0
    for c in samp:
        t0 = time.perf_counter()
        rs_sim(c.to_c(), 10)
        tc += (time.perf_counter() - t0) / 10
    n_mean = sum(c.n for c in cells) / len(cells)
    cpu_proj = tc / sum(c.n for c in samp) * n_mean * len(cells) * B
    line("RG", cells=len(cells), reps_per_cell=B, seconds=t, reps_per_s=len(cells) * B / t,
         cpu_1thread_projected_s=cpu_proj,
         cpu_sample="10 reps of the n=1000 and n=9000 cells, per-sample cost scaled to the grid",
         note="R's own streams (set.seed(1e6+i)); cells run side by side, one MT wave each")


def rstream_hrs():
    import numpy as np
    import torch
    from dcor import hrs
    from oracle import oracle as orc
    age_raw, bmi_raw = hrs.standin_panel(19433, -0.3)
    z = hrs.standardize_panel(age_raw, bmi_raw, lap=np.zeros(4))
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"])
    hrs.eps_sweep(*args, eps_grid=hrs.EPS_GRID[:2], reps=20, rng="R")  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sw = hrs.eps_sweep(*args, rng="R")
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    runs = len(hrs.EPS_GRID) * hrs.R_PER_EPS
    # CPU restatement: the draws of 4 NI + 4 INT runs (estimators excluded), scaled
    n = len(z["age_z"])
    k, m = 4858, 4  # eps = 1.45 geometry; the draw cost is dominated by sample.int and rLap(n)
    t0 = time.perf_counter()
    for r in range(4):
        orc.rs_hrs_ni_draws(10 + 37 * r, n, k, m)
        orc.rs_hrs_int_draws(20 + 41 * r, n, 2000)
    tc = (time.perf_counter() - t0) / 4 * runs
    line("RH", runs_ni=runs, runs_int=runs, seconds=t, runs_per_s=2 * runs / t,
         finite=bool(np.isfinite(sw["runs"]).all()), cpu_draws_only_1thread_projected_s=tc,
         cpu_sample="draws of 4 NI + 4 INT runs (CPU restatement), scaled to the sweep",
         note="each run replays its own set.seed(10 + 37 rep + 1000 idx) / (20 + 41 rep + 1000 idx)")


def dist_grid(name, groups, world, rank, dry_run=False, **extra):
    """One config over the ranks: every rank runs its replicate shard of every (cells, B) group
    (dcor.dist.run_grid_distributed: one batched launch sequence per group, the per-cell
    accumulators all-gathered over RCCL), barrier + synchronize around the timed region, the time
    the max over ranks.  Total replicates are fixed whatever the world size (strong scaling)."""
    import torch
    import torch.distributed as dist
    from dcor.dist import shard
    reps = sum(len(cells) * B for cells, B in groups)
    shards = [[shard(B, r, world) for r in range(world)] for _, B in groups]
    if dry_run:
        if rank == 0:
            print(json.dumps({"config": name, "dry_run": True, "world_formed": dist.get_world_size(),
                              "replicates": reps, "shards": shards, **extra}), flush=True)
        return
    from dcor.dist import run_grid_distributed

    def run():
        return [run_grid_distributed(cells, B) for cells, B in groups]
    run()                                  # warm-up (plans, arenas, RCCL communicator)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    res = run()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    u = sum(grid_units(cells, B) for cells, B in groups)
    n_ok = sum(1 for g in res for (ni, it) in g if ni.n > 0)
    if rank == 0:
        line(name, world_formed=dist.get_world_size(), backend=dist.get_backend(), scaling="strong",
             replicates=reps, seconds=el, reps_per_s=reps / el, roofline_frac_per_gpu=u / el / FP64_PEAK_UNITS / world,
             shards=shards, cells_with_results=n_ok,
             note="one process per GPU: each rank's replicate shard of every cell in one batched launch "
                  "sequence per group, accumulators all-gathered (RCCL); time = max over ranks", **extra)


def hrs_panel(panel="coded"):
    """C5's panel: the coded stand-in (DP-standardised as real-data-sims.R:273-287) or a continuous
    one (every value distinct), and its lambdas."""
    import numpy as np
    from dcor import hrs
    if panel == "coded":
        age_raw, bmi_raw = hrs.standin_panel(19433, -0.3)
        z = hrs.standardize_panel(age_raw, bmi_raw, lap=np.zeros(4))
        return (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"])
    g = np.random.default_rng(2)
    age = np.clip(g.normal(0.0, 1.0, 19433), -2.22, 2.22)
    bmi = -0.19 * age + math.sqrt(1 - 0.19 ** 2) * g.normal(0.0, 1.0, 19433)
    return (age, bmi, 2.22, 2.60)


def dist_hrs(name, world, rank, dry_run, R, mode, panel="coded", sweep=False):
    """The HRS workload over the ranks (real-data-sims.R:411-436): C5-e2e / C5-fused give each rank
    a contiguous range of C5's R replicates (dcor.dist.run_hrs_distributed), the sweep (a19) a
    contiguous range of the flattened (eps, run) space (dcor.dist.eps_sweep_distributed); the records
    are all-gathered in rank order (RCCL).  Strong scaling; time = max over ranks."""
    import torch.distributed as dist
    from dcor.dist import shard, sweep_shard
    if sweep:
        from dcor.hrs import EPS_GRID
        total = len(EPS_GRID) * R
        plan = [sweep_shard(len(EPS_GRID), R, r, world) for r in range(world)]
    else:
        total = R
        plan = [shard(R, r, world) for r in range(world)]
    if dry_run:
        if rank == 0:
            print(json.dumps({"config": name, "dry_run": True, "world_formed": dist.get_world_size(),
                              "replicates": total, "shards": plan}), flush=True)
        return
    import numpy as np
    import torch
    from dcor.dist import eps_sweep_distributed, run_hrs_distributed
    args = hrs_panel(panel)
    if sweep:
        def run():
            return eps_sweep_distributed(*args, reps=R)["runs"].reshape(-1, 6)
    else:
        def run():
            return run_hrs_distributed(*args, 2.0, R, mode=mode, chunk=65536 if mode == "fused" else 8192)
    run()                                   # warm-up (panel, arenas, RCCL communicator)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    res = run()
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    if rank == 0:
        line(name, world_formed=dist.get_world_size(), backend=dist.get_backend(), scaling="strong",
             replicates=total, seconds=el, reps_per_s=total / el, shards=plan, panel=panel, mode=mode,
             finite=bool(np.isfinite(res).all()), rows_gathered=int(res.shape[0]),
             note="one process per GPU: each rank's contiguous replicate range, records all-gathered in rank "
                  "order (RCCL), D2H of every record included; time = max over ranks")


def dist_c5(world, rank, dry_run, R):
    """C5 over the ranks, weak scaling: each rank streams R replicates of its own contiguous range
    (rep_begin = rank R) through the pre-materialised kernel with its noise resident in HBM (c5()'s
    timed launch); value = world R / the max over ranks of the per-launch time."""
    import torch.distributed as dist
    if dry_run:
        if rank == 0:
            print(json.dumps({"config": "C5", "dry_run": True, "world_formed": dist.get_world_size(),
                              "replicates": world * R, "shards": [[r * R, R] for r in range(world)]}), flush=True)
        return
    import torch
    dist.barrier()
    t, per_rep = c5(R, rep_begin=rank * R, emit=False)
    tt = torch.tensor([t], dtype=torch.float64, device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    if rank == 0:
        line("C5", world_formed=dist.get_world_size(), backend=dist.get_backend(), scaling="weak",
             replicates=world * R, seconds=t, reps_per_s=world * R / t, hbm_frac_per_gpu=per_rep * R / t / HBM_PEAK,
             shards=[[r * R, R] for r in range(world)],
             note="one process per GPU, noise resident per rank; time = max over ranks of one "
                  "dcor_premat_subg_panel_launch (best of 5 x 8)")


def main_dist(a, world, rank, local):
    """bench_configs.py under N ranks: C3, C4 and the HRS workload (C5 weak; C5-e2e, C5-fused,
    C5-fused-continuous and the eps sweep HS strong) -- every config that shards."""
    import torch.distributed as dist
    which = a.only.split(",")
    if a.dry_run:
        dist.init_process_group("gloo")
    else:
        import torch
        vis = torch.cuda.device_count()
        if local >= vis:
            sys.exit(f"bench_configs.py: rank {rank}: LOCAL_RANK {local} but {vis} GPU(s) visible "
                     f"(--gpus {world}); refusing to measure fewer")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    formed = dist.get_world_size()
    if formed != world:
        sys.exit(f"bench_configs.py: process group formed {formed} ranks, expected {world}")
    if not a.dry_run:
        import dcor
        dcor._lib.apply_variant_args(a.variant)
    if "C3" in which:
        eps = [tuple(float(v) for v in e.split("x")) for e in a.c3_eps.split(",")] if a.c3_eps else None
        cells = c3_cells(eps)
        dist_grid("C3", [(cells, a.c3_reps)], world, rank, a.dry_run, cells=len(cells), reps_per_cell=a.c3_reps,
                  eps_pairs=eps or C3_EPS)
    if "C5" in which:
        dist_c5(world, rank, a.dry_run, a.c5_R)
    if "C5e" in which:
        dist_hrs("C5-e2e", world, rank, a.dry_run, a.c5e_R, "premat")
    if "C5f" in which:
        dist_hrs("C5-fused", world, rank, a.dry_run, a.c5e_R, "fused")
    if "C5fc" in which:
        dist_hrs("C5-fused-continuous", world, rank, a.dry_run, a.c5e_R, "fused", panel="continuous")
    if "HS" in which:
        dist_hrs("HS", world, rank, a.dry_run, a.hs_R, "premat", sweep=True)
    if "C4" in which:
        ok, small, big, nskip = c4_cells()
        dist_grid("C4", [(small, a.c4_B), (big, a.c4_B_big)], world, rank, a.dry_run, cells=len(ok),
                  cells_skipped_k_lt_1=nskip, reps_per_cell=a.c4_B, reps_per_cell_n1e6=a.c4_B_big,
                  cells_n1e6=len(big))
    others = [w for w in which if w not in ("C3", "C4", "C5", "C5e", "C5f", "C5fc", "HS")]
    if others and rank == 0:
        print(json.dumps({"skipped": others, "reason": "single-GPU configs: run without --gpus"}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C2,C3,C4,VG,SG,C5,C5c,C5e,C5f,C5fc,HS,S,R1,RG,RH")
    ap.add_argument("--c3-reps", type=int, default=100_000)
    ap.add_argument("--c3-eps", default=None, help="subset of C3's eps pairs, e.g. 0.5x0.5,1.5x0.5")
    ap.add_argument("--c4-B", type=int, default=1000)
    ap.add_argument("--c4-B-big", type=int, default=100_000)
    ap.add_argument("--c5-R", type=int, default=8192)
    ap.add_argument("--c5e-R", type=int, default=1_000_000)
    ap.add_argument("--hs-R", type=int, default=200, help="runs per eps of the HRS sweep (real-data-sims.R: R = 200)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="C3, C4, C5, C5e, C5f, C5fc, HS over N ranks (one per GPU); without a launcher's WORLD_SIZE, N rank processes "
                         "are started")
    ap.add_argument("--variant", action="append", default=[], metavar="NAME=VALUE",
                    help="engine implementation switch for A/B runs (dcor_set_variant; repeatable)")
    ap.add_argument("--dry-run", action="store_true",
                    help="with --gpus: form the group over gloo on the CPU and print the shard plan, no GPU")
    a = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus is not None or env_world is not None:
        if env_world is None:
            if a.gpus < 1:
                sys.exit("bench_configs.py: --gpus must be >= 1")
            from bench import spawn_ranks     # the launcher loads no GPU library
            sys.exit(spawn_ranks(a.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
        if a.gpus is not None and a.gpus != int(env_world):
            sys.exit(f"bench_configs.py: --gpus {a.gpus} but the launcher's WORLD_SIZE is {env_world}")
        return main_dist(a, int(env_world), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))
    import torch
    torch.cuda.set_device(0)
    import dcor
    dcor._lib.apply_variant_args(a.variant)
    which = a.only.split(",")
    if "C1" in which: c1()
    if "C2" in which: c2()
    if "C3" in which:
        c3(a.c3_reps, [tuple(float(v) for v in e.split("x")) for e in a.c3_eps.split(",")] if a.c3_eps else None)
    if "C4" in which: c4(a.c4_B, a.c4_B_big)
    if "VG" in which:
        from dcor.sim import vert_cor_grid
        ref_grid("VG", vert_cor_grid())
    if "SG" in which:
        from dcor.sim import subg_grid
        ref_grid("SG", subg_grid())
    if "C5" in which: c5(a.c5_R)
    if "C5c" in which: c5(a.c5_R, panel="continuous")
    if "C5e" in which: c5_e2e(a.c5e_R)
    if "C5f" in which: c5_fused(a.c5e_R)
    if "C5fc" in which: c5_fused(a.c5e_R, panel="continuous")
    if "HS" in which: hrs_sweep(a.hs_R)
    if "S" in which: subg()
    if "R1" in which: rstream_c1()
    if "RG" in which: rstream_grid()
    if "RH" in which: rstream_hrs()


if __name__ == "__main__":
    main()
