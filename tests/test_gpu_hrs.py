"""GPU tests of the HRS replicate driver (real-data-sims.R:345-448, BASELINE config C5) on a
generic stand-in panel: on-device noise streams bit-exact against the oracle's Philox
restatement, every replicate against the oracle estimators, chunk-split invariance, and the
eps sweep summaries."""
import math

import numpy as np
import pytest

from helpers import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def panel():
    import torch
    assert torch.cuda.is_available()
    from dcor import hrs
    age, bmi = hrs.standin_panel(2501, -0.3, seed=5)
    return hrs.standardize_panel(age, bmi, lap=np.array([0.3, -0.2, 0.1, 0.4]))


@pytest.mark.parametrize("eps", [2.0, 0.5])
def test_hrs_replicates_match_oracle(panel, eps):
    _check_against_oracle(panel, eps, R=5, rb=3)


def test_hrs_infinite_panel_value_takes_the_l2_kernel(panel):
    """The coded kernels clip without R's NaN branch because their dictionary is finite: a panel
    with an infinity is not coded (k_panel_dict), and the L2 kernel's results match the oracle."""
    z = dict(panel)
    z["age_z"] = z["age_z"].copy()
    z["bmi_z"] = z["bmi_z"].copy()
    z["age_z"][3] = np.inf
    z["bmi_z"][7] = -np.inf
    _check_against_oracle(z, 2.0, R=2, rb=0)


def _check_against_oracle(z, eps, R, rb):
    from dcor import hrs
    from oracle import oracle as orc
    n = len(z["age_z"])
    res, noise, geo = hrs.hrs_replicates(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps,
                                         R, seed_ni=1010, seed_int=1020, rep_begin=rb, chunk=2,
                                         keep_noise=True)
    k, m = geo["k"], geo["m"]
    for r in range(R):
        rep = rb + r
        np.testing.assert_array_equal(noise["perm"][r], orc.perm(1010, 8, rep, n, k * m))
        for key, seed, site, cnt in (("lap_x", 1010, hrs.SITE_NI_LAP_X, k), ("lap_y", 1010, hrs.SITE_NI_LAP_Y, k),
                                     ("lap_local", 1020, hrs.SITE_INT_LOCAL, n),
                                     ("mix_l", 1020, hrs.SITE_MIX_L, 2000)):
            np.testing.assert_array_equal(noise[key][r], orc.gen_laplace(seed, rep, site, cnt), err_msg=key)
        np.testing.assert_array_equal(noise["mix_z"][r], orc.gen_normals(1020, rep, hrs.SITE_MIX_Z, 2000))
        assert noise["lap_central"][r] == orc.gen_laplace(1020, rep, hrs.SITE_INT_CENTRAL, 1)[0]
        st, ni, km = orc.ni_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_x=z["lambda_age_z"],
                                 lam_y=z["lambda_bmi_z"], perm=noise["perm"][r], lap_x=noise["lap_x"][r],
                                 lap_y=noise["lap_y"][r])
        assert st == 0 and list(km) == [k, m]
        st, it, _ = orc.int_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_s=z["lambda_age_z"],
                                 lam_o=z["lambda_bmi_z"], lam_r=geo["lam_r"], delta=geo["delta"],
                                 lap_local=noise["lap_local"][r], lap_central=noise["lap_central"][r],
                                 mix_z=noise["mix_z"][r], mix_l=noise["mix_l"][r])
        assert st == 0
        assert_close(res[r], np.concatenate([ni, it]), what=f"hrs eps={eps} rep {rep}")


def test_hrs_replicates_match_oracle_c5_size():
    """C5's geometry (n = 19,433, eps = 2 -> m = 2, k = 9,716): the on-device noise and both
    estimators against the oracle, replicates 40 and 41."""
    from dcor import hrs
    from oracle import oracle as orc
    age, bmi = hrs.standin_panel(19_433, -0.3, seed=11)
    z = hrs.standardize_panel(age, bmi, lap=np.array([-0.1, 0.25, 0.05, -0.3]))
    n, eps, rb = 19_433, 2.0, 40
    res, noise, geo = hrs.hrs_replicates(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps,
                                         2, seed_ni=77, seed_int=78, rep_begin=rb, keep_noise=True)
    k, m = geo["k"], geo["m"]
    assert (k, m) == (9716, 2)
    for r in range(2):
        rep = rb + r
        np.testing.assert_array_equal(noise["perm"][r], orc.perm(77, 8, rep, n, k * m))
        np.testing.assert_array_equal(noise["lap_local"][r], orc.gen_laplace(78, rep, hrs.SITE_INT_LOCAL, n))
        st, ni, _ = orc.ni_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_x=z["lambda_age_z"],
                                lam_y=z["lambda_bmi_z"], perm=noise["perm"][r], lap_x=noise["lap_x"][r],
                                lap_y=noise["lap_y"][r])
        st2, it, _ = orc.int_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_s=z["lambda_age_z"],
                                  lam_o=z["lambda_bmi_z"], lam_r=geo["lam_r"], delta=geo["delta"],
                                  lap_local=noise["lap_local"][r], lap_central=noise["lap_central"][r],
                                  mix_z=noise["mix_z"][r], mix_l=noise["mix_l"][r])
        assert st == 0 and st2 == 0
        assert_close(res[r], np.concatenate([ni, it]), what=f"hrs C5 size rep {rep}")


def test_hrs_replicates_split_invariant(panel):
    from dcor import hrs
    z = panel
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 1.05)
    whole = hrs.hrs_replicates(*args, 9, chunk=9)
    parts = np.concatenate([hrs.hrs_replicates(*args, 4, chunk=3),
                            hrs.hrs_replicates(*args, 5, rep_begin=4, chunk=5)])
    np.testing.assert_array_equal(whole.view(np.int64), parts.view(np.int64))


@pytest.mark.parametrize("kind,n", [("coded", 3003), ("continuous", 3003), ("continuous", 3001)])
def test_premat_replicate_independent_of_row_position(kind, n):
    """Odd n (odd k): every other noise row of a launch starts 8 B off a 16-B boundary.  INT sample
    pairs and NI batch pairs are formed by index whatever the row's alignment, so a replicate run as
    row 0 of its own launch equals the same replicate run as row 1..5 of a six-row launch, bit for
    bit -- on the coded kernel (k odd), the L2-gather kernel (k odd) and the tiled kernel (k even)."""
    from dcor import hrs
    if kind == "coded":
        age, bmi = hrs.standin_panel(n, -0.3, seed=7)
        z = hrs.standardize_panel(age, bmi, lap=np.array([0.1, 0.2, -0.3, 0.05]))
    else:
        z = _continuous(n, seed=n)
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0)
    whole = hrs.hrs_replicates(*args, 6, rep_begin=1, chunk=6)
    ones = np.concatenate([hrs.hrs_replicates(*args, 1, rep_begin=1 + r, chunk=1) for r in range(6)])
    np.testing.assert_array_equal(whole.view(np.int64), ones.view(np.int64))


def test_eps_sweep_summaries(panel):
    from dcor import hrs
    z = panel
    out = hrs.eps_sweep(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps_grid=(0.25, 2.45),
                        reps=4)
    assert out["runs"].shape == (2, 4, 6)
    for s, runs in zip(out["ni_mean"], out["runs"]):
        assert s["method"] == "NI"
        assert math.isclose(s["rho_hat_mean"], float(np.mean(runs[:, 0])), rel_tol=0, abs_tol=0)
        assert math.isclose(s["ci_low_q10"], float(np.quantile(runs[:, 1], 0.1)), rel_tol=0, abs_tol=0)
    for s, runs in zip(out["int_mean"], out["runs"]):
        assert s["method"] == "INT" and s["ci_low_mean"] <= s["ci_high_mean"]  # rho_hat is not clipped
        assert math.isclose(s["ci_high_q90"], float(np.quantile(runs[:, 5], 0.9)), rel_tol=0, abs_tol=0)
    assert [round(e, 2) for e in hrs.EPS_GRID][:3] == [0.25, 0.35, 0.45] and len(hrs.EPS_GRID) == 23


@pytest.mark.parametrize("kind", ["coded", "continuous"])
def test_sweep_segments_equal_per_eps_calls(panel, kind):
    """hrs.sweep_segments (one encoded panel, the native launch chain dcor_hrs_sweep_launch with
    its one-launch noise kernel, optionally over HIP streams, one wait) equals the host-driven
    chain (hrs_replicates with keep_noise: the seven noise launches from Python) per segment with
    the sweep's keys, byte for byte; segments start mid-eps (rep_begin > 0) as a rank's shard does."""
    from dcor import hrs
    z = panel if kind == "coded" else _continuous(2501, seed=9)
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"])
    grid = (0.25, 1.05, 2.45)
    segs = [(0, 3, 5), (1, 0, 7), (2, 2, 1), (0, 8, 2), (1, 7, 3)]
    want = np.concatenate([hrs.hrs_replicates(*args, grid[e], c, seed_ni=10 + 1000 * (e + 1),
                                              seed_int=20 + 1000 * (e + 1), rep_begin=r0, keep_noise=True)[0]
                           for e, r0, c in segs])
    for streams in (1, 4):
        got = hrs.sweep_segments(*args, grid, segs, streams=streams)
        np.testing.assert_array_equal(got.view(np.int64), want.view(np.int64), err_msg=f"streams={streams}")
    sw = hrs.eps_sweep(*args, eps_grid=grid, reps=4)
    one = np.stack([hrs.hrs_replicates(*args, e, 4, seed_ni=10 + 1000 * i, seed_int=20 + 1000 * i)
                    for i, e in enumerate(grid, start=1)])
    np.testing.assert_array_equal(sw["runs"].view(np.int64), one.view(np.int64))


def test_sweep_segments_past_one_launch(panel):
    """A segment longer than one launch chain (8192 runs) splits like the host-driven chunks."""
    from dcor import hrs
    z = panel
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"])
    got = hrs.sweep_segments(*args, (2.0,), [(0, 5, 8195)], streams=2)
    want = hrs.hrs_replicates(*args, 2.0, 8195, seed_ni=1010, seed_int=1020, rep_begin=5, keep_noise=True)[0]
    np.testing.assert_array_equal(got.view(np.int64), want.view(np.int64))


def test_sweep_launch_checks_every_segment_first(panel):
    """dcor_hrs_sweep_launch rejects a bad segment (eps <= 0, negative counts, a replicate range past
    2^32) or a bad base (not the panel's n, nsim 0, delta 0, not HRS) before it enqueues anything:
    the output rows stay untouched; an empty segment list or zero-run segments are no-ops."""
    import ctypes as C

    import torch
    from dcor import _lib
    z = panel
    X = torch.as_tensor(z["age_z"], device="cuda")
    Y = torch.as_tensor(z["bmi_z"], device="cuda")
    n = int(X.shape[0])
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    pn = C.c_void_p()
    _lib.check(_lib.lib.dcor_panel_create(C.c_void_p(X.data_ptr()), C.c_void_p(Y.data_ptr()), n, sp, C.byref(pn)))
    try:
        out = torch.full((8, 6), 7.0, dtype=torch.float64, device="cuda")
        base = _lib.PrematSubg(n=n, eta1=1.0, eta2=1.0, alpha=0.05, hrs=1, lam_x=z["lambda_age_z"],
                               lam_y=z["lambda_bmi_z"], lam_s=z["lambda_age_z"], lam_o=z["lambda_bmi_z"],
                               delta=1.0 / n, nsim=2000, X=X.data_ptr(), Y=Y.data_ptr())
        good = _lib.HrsSegment(eps=2.0, seed_ni=1, seed_int=2, rep_begin=0, reps=4, out_row=0)
        for bad in (dict(eps=0.0), dict(eps=-1.0), dict(reps=-1), dict(rep_begin=-2), dict(out_row=-1)):
            seg = _lib.HrsSegment(**{**dict(eps=1.0, seed_ni=1, seed_int=2, rep_begin=0, reps=4, out_row=4), **bad})
            arr = (_lib.HrsSegment * 2)(good, seg)
            st = _lib.lib.dcor_hrs_sweep_launch(C.byref(base), pn, arr, 2, C.c_void_p(out.data_ptr()), sp)
            assert st == _lib.DCOR_EINVAL, bad
        arr = (_lib.HrsSegment * 1)(good)
        for field, value in (("n", n - 1), ("nsim", 0), ("delta", 0.0), ("hrs", 0)):
            other = _lib.PrematSubg.from_buffer_copy(bytes(base))
            setattr(other, field, value)
            st = _lib.lib.dcor_hrs_sweep_launch(C.byref(other), pn, arr, 1, C.c_void_p(out.data_ptr()), sp)
            assert st == _lib.DCOR_EINVAL, field
        far = (_lib.HrsSegment * 1)(_lib.HrsSegment(eps=2.0, seed_ni=1, seed_int=2, rep_begin=2**32 - 2, reps=4))
        assert _lib.lib.dcor_hrs_sweep_launch(C.byref(base), pn, far, 1, C.c_void_p(out.data_ptr()), sp) == _lib.DCOR_EINVAL
        torch.cuda.synchronize()
        assert bool((out == 7.0).all())
        empty = (_lib.HrsSegment * 1)(_lib.HrsSegment(eps=2.0, reps=0, out_row=0))
        _lib.check(_lib.lib.dcor_hrs_sweep_launch(C.byref(base), pn, empty, 0, C.c_void_p(out.data_ptr()), sp))
        _lib.check(_lib.lib.dcor_hrs_sweep_launch(C.byref(base), pn, empty, 1, C.c_void_p(out.data_ptr()), sp))
        torch.cuda.synchronize()
        assert bool((out == 7.0).all())
    finally:
        _lib.lib.dcor_panel_destroy(pn)


@pytest.mark.parametrize("kind", ["coded", "continuous"])
def test_native_chain_equals_host_chain(panel, kind):
    """hrs_replicates' native chain (rng='philox', no keep_noise) equals the host-driven chain
    (keep_noise=True: perm + six draw launches from Python, each checked against the oracle in
    _check_against_oracle) byte for byte, chunked or not."""
    from dcor import hrs
    z = panel if kind == "coded" else _continuous(2501, seed=4)
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 0.85)
    host = hrs.hrs_replicates(*args, 7, seed_ni=5, seed_int=6, rep_begin=2, keep_noise=True)[0]
    for chunk in (3, 8192):
        nat = hrs.hrs_replicates(*args, 7, seed_ni=5, seed_int=6, rep_begin=2, chunk=chunk)
        np.testing.assert_array_equal(nat.view(np.int64), host.view(np.int64), err_msg=f"chunk={chunk}")


def test_panel_pipelined_halves_bitexact(panel):
    """Large coded-panel launches split into two stream-pipelined halves; the result must
    equal the single-stream launch bit for bit."""
    import os
    from dcor import hrs
    z = panel
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0, 4100)
    serial = hrs.hrs_replicates(*args, chunk=4100)
    from dcor import _lib
    with _lib.variants(DCOR_PREMAT_PIPELINE="1"):
        piped = hrs.hrs_replicates(*args, chunk=4100)
    np.testing.assert_array_equal(piped.view(np.int64), serial.view(np.int64))
    assert np.isfinite(piped).all()


# ------------------------------------------------------- R-stream runs (f4 + a19)
@pytest.mark.parametrize("eps,idx", [(2.0, 18), (0.35, 2)])
def test_hrs_r_streams_match_oracle(panel, eps, idx):
    """rng='R': run rep draws after set.seed(10 + 37 rep + 1000 idx) / set.seed(20 + 41 rep +
    1000 idx) (real-data-sims.R:404, 423): sample.int, rLap and mixquant bit-exact against the
    CPU restatement, estimates within 1e-12."""
    from dcor import hrs
    from oracle import oracle as orc
    z = panel
    n = len(z["age_z"])
    R, rb = 4, 6
    res, noise, geo = hrs.hrs_replicates(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps,
                                         R, rep_begin=rb, chunk=3, keep_noise=True, rng="R", eps_idx=idx)
    k, m = geo["k"], geo["m"]
    sn, si = hrs.r_seeds(idx, R, rb)
    assert sn[0] == 10 + 37 * (rb + 1) + 1000 * idx and si[0] == 20 + 41 * (rb + 1) + 1000 * idx
    for r in range(R):
        perm, lx, ly = orc.rs_hrs_ni_draws(int(sn[r]), n, k, m)
        np.testing.assert_array_equal(noise["perm"][r], perm)
        np.testing.assert_array_equal(noise["lap_x"][r], lx)
        np.testing.assert_array_equal(noise["lap_y"][r], ly)
        ll, lc, mz, ml = orc.rs_hrs_int_draws(int(si[r]), n, 2000)
        np.testing.assert_array_equal(noise["lap_local"][r], ll)
        assert noise["lap_central"][r] == lc
        np.testing.assert_array_equal(noise["mix_z"][r], mz)
        np.testing.assert_array_equal(noise["mix_l"][r], ml)
        st, ni, _ = orc.ni_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_x=z["lambda_age_z"],
                                lam_y=z["lambda_bmi_z"], perm=perm, lap_x=lx, lap_y=ly)
        st2, it, _ = orc.int_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_s=z["lambda_age_z"],
                                  lam_o=z["lambda_bmi_z"], lam_r=geo["lam_r"], delta=geo["delta"],
                                  lap_local=ll, lap_central=lc, mix_z=mz, mix_l=ml)
        assert st == 0 and st2 == 0
        assert_close(res[r], np.concatenate([ni, it]), what=f"R-stream hrs eps={eps} run {rb + r + 1}")


def test_hrs_r_stream_sample_int_is_a_permutation(panel):
    import ctypes as C

    import torch
    from dcor import _lib
    n, k, m, runs = 20000, 9000, 2, 3
    perm = torch.empty((runs, k * m), dtype=torch.int32, device="cuda")
    lx = torch.empty((runs, k), dtype=torch.float64, device="cuda")
    ly = torch.empty_like(lx)
    seeds = np.array([1, 42, 123], dtype=np.int32)
    P = lambda t: C.c_void_p(t.data_ptr())
    _lib.check(_lib.lib.dcor_rstream_hrs_draws(n, k, m, 2000, runs, seeds.ctypes.data_as(C.POINTER(C.c_int32)),
                                               None, P(perm), P(lx), P(ly), None, None, None, None, None))
    got = perm.cpu().numpy()
    from oracle import oracle as orc
    for r in range(runs):
        assert len(np.unique(got[r])) == k * m and got[r].min() >= 0 and got[r].max() < n
        np.testing.assert_array_equal(got[r], orc.rs_sample_int(int(seeds[r]), n, k * m))
    # R: set.seed(1); sample(10) = 9 4 7 1 2 5 3 10 6 8 (tests/golden/r_known_values.json)
    p10 = torch.empty((1, 10), dtype=torch.int32, device="cuda")
    l1 = torch.empty((1, 5), dtype=torch.float64, device="cuda")
    one = np.array([1], dtype=np.int32)
    _lib.check(_lib.lib.dcor_rstream_hrs_draws(10, 5, 2, 2000, 1, one.ctypes.data_as(C.POINTER(C.c_int32)),
                                               None, P(p10), P(l1), P(l1), None, None, None, None, None))
    assert list(p10.cpu().numpy()[0] + 1) == [9, 4, 7, 1, 2, 5, 3, 10, 6, 8]


# ------------------------------------------------ fused HRS (noise drawn in the kernel)
@pytest.mark.parametrize("n,eps,reps,rb", [(2501, 2.0, 37, 0), (2501, 2.0, 9, 1001), (2501, 0.55, 11, 5),
                                           (2501, 1.05, 7, 0), (2500, 2.0, 6, 2), (19433, 2.0, 5, 17)])
def test_hrs_fused_equals_premat(n, eps, reps, rb):
    """dcor_hrs_fused_launch draws the HRS driver's Philox streams in the kernel: every
    replicate equals the pre-materialised pipeline's (whose noise the other tests pin
    bit-exact against the oracle) within the estimator tolerance; odd / even n, m = 2 and
    m > 2 batches, a replicate offset."""
    from dcor import hrs
    age, bmi = hrs.standin_panel(n, -0.3, seed=5)
    z = hrs.standardize_panel(age, bmi, lap=np.array([0.3, -0.2, 0.1, 0.4]))
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps, reps)
    pm = hrs.hrs_replicates(*args, rep_begin=rb)
    fu = hrs.hrs_replicates(*args, rep_begin=rb, mode="fused")
    assert np.isfinite(fu).all()
    for r in range(reps):
        assert_close(fu[r], pm[r], what=f"fused vs premat n={n} eps={eps} rep {rb + r}")


def test_hrs_fused_split_invariant(panel):
    from dcor import hrs
    z = panel
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0)
    whole = hrs.hrs_replicates(*args, 10, chunk=10, mode="fused")
    parts = np.concatenate([hrs.hrs_replicates(*args, 3, chunk=3, mode="fused"),
                            hrs.hrs_replicates(*args, 7, rep_begin=3, chunk=4, mode="fused")])
    np.testing.assert_array_equal(whole.view(np.int64), parts.view(np.int64))


def _continuous(n, seed=1):
    """A panel no dictionary codes: every value distinct (standardised normal draws)."""
    g = np.random.default_rng(seed)
    x = g.standard_normal(n)
    y = -0.3 * x + math.sqrt(1 - 0.09) * g.standard_normal(n)
    return {"age_z": x, "bmi_z": y, "lambda_age_z": 2.2, "lambda_bmi_z": 2.6}


@pytest.mark.parametrize("n,eps,reps,rb", [(3001, 2.0, 9, 0), (3000, 0.55, 5, 11), (19433, 2.0, 4, 40)])
def test_hrs_fused_continuous_panel_matches_oracle(n, eps, reps, rb):
    """mode='fused' on a panel with no dictionary (k_hrs_fused_l2): every replicate against the
    oracle estimators fed the oracle's own Philox restatement of the same streams."""
    from dcor import api, hrs
    from oracle import oracle as orc
    z = _continuous(n)
    fu = hrs.hrs_replicates(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps, reps,
                            seed_ni=1010, seed_int=1020, rep_begin=rb, mode="fused")
    k, m = api.batch_geometry(n, eps, eps, "subG", hrs=True)
    delta = 1.0 / n
    lam_r = api.lambda_receiver_from_noise(z["lambda_age_z"], z["lambda_bmi_z"], eps, delta)
    for r in range(reps):
        rep = rb + r
        st, ni, _ = orc.ni_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_x=z["lambda_age_z"],
                                lam_y=z["lambda_bmi_z"], perm=orc.perm(1010, 8, rep, n, k * m),
                                lap_x=orc.gen_laplace(1010, rep, hrs.SITE_NI_LAP_X, k),
                                lap_y=orc.gen_laplace(1010, rep, hrs.SITE_NI_LAP_Y, k))
        st2, it, _ = orc.int_subg(z["age_z"], z["bmi_z"], eps, eps, hrs=1, lam_s=z["lambda_age_z"],
                                  lam_o=z["lambda_bmi_z"], lam_r=lam_r, delta=delta,
                                  lap_local=orc.gen_laplace(1020, rep, hrs.SITE_INT_LOCAL, n),
                                  lap_central=orc.gen_laplace(1020, rep, hrs.SITE_INT_CENTRAL, 1)[0],
                                  mix_z=orc.gen_normals(1020, rep, hrs.SITE_MIX_Z, 2000),
                                  mix_l=orc.gen_laplace(1020, rep, hrs.SITE_MIX_L, 2000))
        assert st == 0 and st2 == 0
        assert_close(fu[r], np.concatenate([ni, it]), what=f"fused continuous n={n} eps={eps} rep {rep}")


def test_hrs_fused_l2_kernel_equals_coded_kernel(panel):
    """On a codable panel the uncoded kernel (DCOR_HRS_FUSED_L2=1) gathers the same clipped values
    the coded kernel reads from its dictionaries, in the same order: identical bits."""
    from dcor import _lib, hrs
    z = panel
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0, 23)
    coded = hrs.hrs_replicates(*args, rep_begin=5, mode="fused")
    with _lib.variants(DCOR_HRS_FUSED_L2="1"):
        l2 = hrs.hrs_replicates(*args, rep_begin=5, mode="fused")
    np.testing.assert_array_equal(l2.view(np.int64), coded.view(np.int64))


def test_hrs_fused_large_uncoded_panel_materialises():
    """n > 65536 with no dictionary: the fused entry materialises the same streams and runs the
    pre-materialised kernels, so its replicates equal mode='premat' exactly."""
    from dcor import hrs
    z = _continuous(70001, seed=3)
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0, 3)
    fu = hrs.hrs_replicates(*args, rep_begin=2, mode="fused")
    pm = hrs.hrs_replicates(*args, rep_begin=2)
    np.testing.assert_array_equal(fu.view(np.int64), pm.view(np.int64))


_TILED_CASES = ((1001, 2.0, 5, 3), (19433, 2.0, 5, 17), (30001, 2.0, 3, 0), (19433, 0.5, 2, 0))


def _premat_continuous_runs():
    from dcor import hrs
    out = {}
    for n, eps, reps, rb in _TILED_CASES:
        z = _continuous(n, seed=n)
        out[f"{n}_{eps}"] = hrs.hrs_replicates(z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps,
                                               reps, seed_ni=31, seed_int=32, rep_begin=rb)
    return out


def test_premat_tiled_kernel_matches_l2_kernel():
    """Continuous panels, m = 2 (and one m > 2 case, which keeps the L2-gather kernel).  The
    512-thread tiled kernel (DCOR_TILED_VARIANT=0) returns the L2-gather kernel's bits (DCOR_TILED=0:
    same work split, same pair-grouped sums) whether its INT sums run in k_premat_subg_int on the
    same stream (default), on the auxiliary stream (DCOR_TILED_INT=2) or inside the tiled kernel
    (DCOR_TILED_INT=0); the default 1024-thread variant splits the NI batch pairs over 1024 threads
    and agrees within the estimator tolerance.  n = 1001 is one tile, 19,433 four (512 threads) or
    two (1024); 30,001 takes two rounds of batch pairs in both variants, 19,433 in the 512-thread
    one; odd n puts every other replicate's noise row off a 16-B boundary (the head-sample path).
    The estimators against the oracle on this path: test_gpu_more.py::test_premat_subg_hrs_shared_panel."""
    from dcor import _lib
    got = _premat_continuous_runs()
    runs = {}
    variants = (("l2", {"DCOR_TILED": "0"}), ("v0", {"DCOR_TILED_VARIANT": "0"}),
                ("v0_aux", {"DCOR_TILED_VARIANT": "0", "DCOR_TILED_INT": "2"}),
                ("v0_in", {"DCOR_TILED_VARIANT": "0", "DCOR_TILED_INT": "0"}))
    for name, over in variants:
        with _lib.variants(**over):
            runs[name] = _premat_continuous_runs()
    for key, v in got.items():
        assert np.isfinite(v).all()
        for name in ("v0", "v0_aux", "v0_in"):
            np.testing.assert_array_equal(runs[name][key].view(np.int64), runs["l2"][key].view(np.int64),
                                          err_msg=f"{key}: 512-thread tiled ({name}) vs L2 kernel")
        for r in range(len(v)):
            assert_close(v[r], runs["l2"][key][r], what=f"{key} rep {r} default vs L2 kernel")


def test_premat_tiled_workgroup_runs_many_replicates():
    """One launch with more replicates than the tiled kernel's resident workgroups: each
    workgroup then runs several replicates in turn, starting each on the panel tile its previous
    replicate left in LDS (every other sweep reversed), and the INT kernel groups four replicates
    per workgroup with a short last group.  Sampled rows equal the same replicates run one per
    launch (a fresh workgroup, every tile filled), bit for bit, and the oracle-checked 512-thread
    variant's rows within the estimator tolerance."""
    from dcor import hrs
    z = _continuous(3001, seed=11)
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], 2.0)
    R = 1203                     # > 256 CUs x 1 workgroup, and R % 4 == 3
    whole = hrs.hrs_replicates(*args, R, rep_begin=5, chunk=R)
    assert np.isfinite(whole).all()
    for r in (0, 1, 255, 256, 257, 511, 767, 1023, 1200, 1201, 1202):
        one = hrs.hrs_replicates(*args, 1, rep_begin=5 + r, chunk=1)
        np.testing.assert_array_equal(whole[r:r + 1].view(np.int64), one.view(np.int64), err_msg=f"row {r}")
    from dcor import _lib
    with _lib.variants(DCOR_TILED_VARIANT="0"):
        v0 = hrs.hrs_replicates(*args, R, rep_begin=5, chunk=R)
    for r in range(0, R, 97):
        assert_close(whole[r], v0[r], what=f"row {r}: default vs 512-thread tiled kernel")


@pytest.mark.parametrize("off", [1, 2, 3])
def test_premat_tiled_kernel_independent_of_buffer_alignment(off):
    """The uncoded-panel dispatch depends on the geometry only: the caller's index and NI-noise
    arrays placed `off` elements past a 16-B boundary (4-B / 8-B aligned) run the same tiled kernel,
    reading rows element by element, and return the aligned launch's bits."""
    import ctypes as C

    import torch
    from dcor import _lib, api, hrs
    z = _continuous(3001, seed=5)
    eps, R = 2.0, 5
    args = (z["age_z"], z["bmi_z"], z["lambda_age_z"], z["lambda_bmi_z"], eps)
    ref, noise, geo = hrs.hrs_replicates(*args, R, seed_ni=41, seed_int=42, keep_noise=True)
    k, m = geo["k"], geo["m"]
    assert m == 2 and k % 2 == 0
    n = len(z["age_z"])

    def dev(a, dtype, shift):
        a = np.ascontiguousarray(a)
        t = torch.empty(a.size + 4, dtype=dtype, device="cuda")
        assert t.data_ptr() % 16 == 0
        v = t[shift:shift + a.size]
        v.copy_(torch.as_tensor(a.ravel()))
        return v
    perm = dev(noise["perm"], torch.int32, off)
    lx = dev(noise["lap_x"], torch.float64, 1)
    ly = dev(noise["lap_y"], torch.float64, 1)
    ll = dev(noise["lap_local"], torch.float64, 0)
    lc = dev(noise["lap_central"], torch.float64, 0)
    mz = dev(noise["mix_z"], torch.float64, 0)
    ml = dev(noise["mix_l"], torch.float64, 0)
    X = torch.as_tensor(z["age_z"], device="cuda")
    Y = torch.as_tensor(z["bmi_z"], device="cuda")
    out = torch.empty((R, 6), dtype=torch.float64, device="cuda")
    P = lambda t: C.c_void_p(t.data_ptr())
    pn = C.c_void_p()
    _lib.check(_lib.lib.dcor_panel_create(P(X), P(Y), n, None, C.byref(pn)))
    try:
        d = _lib.PrematSubg(n=n, reps=R, eps1=eps, eps2=eps, eta1=1.0, eta2=1.0, alpha=0.05, hrs=1,
                            lam_x=args[2], lam_y=args[3], lam_s=args[2], lam_o=args[3], lam_r=geo["lam_r"],
                            delta=geo["delta"], nsim=2000, X=X.data_ptr(), Y=Y.data_ptr(), xy_stride=0,
                            perm=perm.data_ptr(), lap_ni_x=lx.data_ptr(), lap_ni_y=ly.data_ptr(),
                            lap_local=ll.data_ptr(), lap_central=lc.data_ptr(), mix_z=mz.data_ptr(),
                            mix_l=ml.data_ptr())
        _lib.check(_lib.lib.dcor_premat_subg_panel_launch(C.byref(d), pn, P(out), None))
        got = out.cpu().numpy()
    finally:
        _lib.lib.dcor_panel_destroy(pn)
    np.testing.assert_array_equal(got.view(np.int64), ref.view(np.int64))
