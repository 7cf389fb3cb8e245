"""GPU tests beyond single-call parity: golden fixtures, batched device-pointer
pre-materialised launches (per-replicate strides, shared HRS panel), NA / edge
semantics, accumulation kernel, full-size invariants and an independent-RNG
Monte-Carlo coverage comparison."""
import ctypes as C
import math
import os

import numpy as np
import pytest

from helpers import assert_close, sign_case, subg_case, unit_laplace

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "explicit_cases.npz")


@pytest.fixture(scope="module")
def dc():
    import torch
    assert torch.cuda.is_available()
    import dcor
    return dcor


@pytest.fixture(scope="module")
def orc():
    from oracle import oracle
    return oracle


def _t(a, dtype=None):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a), device="cuda", dtype=dtype)


# -------------------------------------------------------------- golden files
def test_golden_gpu(dc):
    d = np.load(GOLD, allow_pickle=False)
    for i in range(int(d["n_sign"][0])):
        p = f"sign{i}_"
        n, e1, e2, lz = d[p + "scalars"]
        X, Y = d[p + "X"], d[p + "Y"]
        if not np.all(np.isnan(d[p + "ni"])):
            got = dc.ci_NI_signbatch(X, Y, e1, e2, noise={"lap_sc": d[p + "lap_ni_sc"], "lap_x": d[p + "lap_x"],
                                                          "lap_y": d[p + "lap_y"]})
            assert_close([got["rho_hat"], *got["ci"]], d[p + "ni"], what=p + "ni")
        for md in range(3):
            got = dc.ci_INT_signflip(X, Y, e1, e2, mode=md, noise={
                "lap_sc": d[p + "lap_int_sc"], "flips": d[p + "flips"], "lap_z": lz,
                "mix_z": d[p + "mix_z"], "mix_l": d[p + "mix_l"]})
            assert_close([got["rho_hat"], *got["ci"]], d[p + "int"][md], what=p + f"int{md}")
    for i in range(int(d["n_subg"][0])):
        p = f"subg{i}_"
        n, e1, e2, lc, hrs, lx, ly = d[p + "scalars"]
        hrs = bool(hrs)
        got = dc.correlation_NI_subG(d[p + "X"], d[p + "Y"], e1, e2, hrs=hrs,
                                     lambda_X=lx if hrs else None, lambda_Y=ly if hrs else None,
                                     perm=d[p + "perm"] if hrs else None,
                                     noise={"lap_x": d[p + "lap_x"], "lap_y": d[p + "lap_y"]})
        assert_close([got["rho_hat"], *got["ci"]], d[p + "ni"], what=p + "ni")
        got = dc.ci_INT_subG(d[p + "X"], d[p + "Y"], e1, e2, hrs=hrs,
                             lambda_sender=lx if hrs else None, lambda_other=ly if hrs else None,
                             noise={"lap_local": d[p + "lap_local"], "lap_central": lc,
                                    "mix_z": d[p + "mix_z"], "mix_l": d[p + "mix_l"]})
        assert_close([got["rho_hat"], *got["ci"]], d[p + "int"], what=p + "int")
    for j in range(12):
        c, want = d[f"mq{j}_c"]
        got = dc.mixquant(c, 0.975, z=d[f"mq{j}_z"], l=d[f"mq{j}_l"])
        assert got == want or (math.isnan(got) and math.isnan(want))
    for j in range(6):
        eps, L = d[f"ps{j}_par"]
        assert_close(dc.priv_standardize(d[f"ps{j}_v"], eps, L, lap=d[f"ps{j}_lap"]), d[f"ps{j}_out"])
        s = dc.dp_sd(d[f"sd{j}_x"], 45.0, 90.0, 0.1, 0.1, lap=d[f"sd{j}_lap"])
        assert_close([s["mean"], s["sd"]], d[f"sd{j}_out"])


# ------------------------------------------------ batched device launches
def test_premat_sign_batch_device(dc, orc):
    import torch
    from dcor import _lib
    R, n, e1, e2 = 6, 5000, 1.5, 0.5
    g = np.random.default_rng(42)
    cases = [sign_case(g, n, e1, e2, rho=r) for r in np.linspace(-0.8, 0.8, R)]
    k = cases[0]["k"]
    fw = (n + 31) // 32
    flips = np.zeros((R, fw), dtype=np.uint32)
    for r, cs in enumerate(cases):
        for i in np.nonzero(cs["flips"])[0]:
            flips[r, i >> 5] |= np.uint32(1 << (i & 31))
    t = {key: _t(np.stack([cs[key] for cs in cases])) for key in
         ("X", "Y", "lap_ni_sc", "lap_x", "lap_y", "lap_int_sc", "mix_z", "mix_l")}
    t["lap_z"] = _t(np.array([cs["lap_z"] for cs in cases]))
    t["flips"] = _t(flips.view(np.int32))
    d = _lib.PrematSign(n=n, reps=R, eps1=e1, eps2=e2, alpha=0.05, normalise=1, ci_mode=0, nsim=1000,
                        X=t["X"].data_ptr(), Y=t["Y"].data_ptr(), xy_stride=n,
                        lap_ni_sc=t["lap_ni_sc"].data_ptr(), lap_ni_x=t["lap_x"].data_ptr(),
                        lap_ni_y=t["lap_y"].data_ptr(), lap_int_sc=t["lap_int_sc"].data_ptr(),
                        flips=t["flips"].data_ptr(), lap_z=t["lap_z"].data_ptr(),
                        mix_z=t["mix_z"].data_ptr(), mix_l=t["mix_l"].data_ptr())
    out = torch.empty((R, 6), dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.dcor_premat_sign_launch(C.byref(d), C.c_void_p(out.data_ptr()), None))
    got = out.cpu().numpy()
    for r, cs in enumerate(cases):
        _, ni = orc.ci_ni_signbatch(cs["X"], cs["Y"], e1, e2, 0.05, 1, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
        _, it, _ = orc.ci_int_signflip(cs["X"], cs["Y"], e1, e2, 0.05, 0, 1, cs["lap_int_sc"], cs["flips"],
                                       cs["lap_z"], cs["mix_z"], cs["mix_l"])
        assert_close(got[r], np.concatenate([ni, it]), what=f"rep {r}")


def _hrs_panel(kind, n, g):
    """Shared HRS-like panels: 'continuous' (every value distinct: L2-gather kernel), 'coded'
    (integer ages, one-decimal BMI like the real wave-2 panel: dictionary-coded LDS kernel),
    'd256' / 'd257' (exactly 256 / 257 distinct values in X: the dictionary boundary)."""
    if kind == "continuous":
        age = np.clip(g.normal(0.0, 1.0, n), -2.2, 2.2)
        bmi = -0.19 * age + math.sqrt(1 - 0.19 ** 2) * g.normal(0.0, 1.0, n)
        return age, bmi
    if kind == "coded":
        a = np.clip(np.round(g.normal(65.0, 10.0, n)), 23, 103)
        b = np.round(np.clip(g.normal(27.0, 5.0, n) - 0.05 * (a - 65.0), 12.6, 92.2), 1)
        a = (np.clip(a, 45, 90) - 66.1) / 9.7     # standardize_dp (real-data-sims.R:87-90)
        b = (np.clip(b, 15, 35) - 26.9) / 4.6
        return a, b
    d = 256 if kind == "d256" else 257
    vals = np.linspace(-2.0, 2.0, d)
    a = vals[np.arange(n) % d]
    g.shuffle(a)
    b = np.round(g.normal(0.0, 1.0, n), 1)
    return a, b


@pytest.mark.parametrize("kind,n,eps", [("continuous", 19433, 2.0), ("coded", 19433, 2.0),
                                        ("coded", 19433, 0.5), ("coded", 1001, 2.0),
                                        ("coded", 1002, 2.0), ("coded", 1003, 2.0),
                                        ("d256", 5000, 2.0), ("d257", 5000, 2.0),
                                        ("continuous", 3000, 0.5), ("continuous", 4999, 2.0),
                                        ("continuous-dup", 19433, 2.0), ("continuous-dup", 1001, 2.0)])
def test_premat_subg_hrs_shared_panel(dc, orc, kind, n, eps):
    """HRS mode: one shared (X, Y) panel (stride 0), per-replicate perms and noise; the
    dictionary-coded kernel (few distinct values) and the uncoded kernels (tiled for m = 2,
    L2-gather otherwise).  'continuous-dup': replicates 1 and 3 draw their batches WITH
    replacement (the ABI takes any index rows, not only sample.int's): a repeated sample index
    must be read twice, whatever the kernel."""
    import torch
    from dcor import _lib
    R = 5
    g = np.random.default_rng(7)
    dup = kind.endswith("-dup")
    kind = kind.replace("-dup", "")
    age, bmi = _hrs_panel(kind, n, g)
    k, m = dc.api.batch_geometry(n, eps, eps, "subG", hrs=True)
    perms = np.stack([g.permutation(n)[: k * m] for _ in range(R)]).astype(np.int32)
    if dup:
        perms[1] = g.integers(0, n, k * m)
        perms[3] = perms[0]
        perms[3][5] = perms[3][9]
    lx, ly = unit_laplace(g, (R, k)), unit_laplace(g, (R, k))
    ll, lc = unit_laplace(g, (R, n)), unit_laplace(g, R)
    mz, ml = g.standard_normal((R, 2000)), unit_laplace(g, (R, 2000))
    T = {"X": _t(age), "Y": _t(bmi), "perm": _t(perms), "lx": _t(lx), "ly": _t(ly), "ll": _t(ll),
         "lc": _t(lc), "mz": _t(mz), "ml": _t(ml)}
    d = _lib.PrematSubg(n=n, reps=R, eps1=eps, eps2=eps, eta1=1.0, eta2=1.0, alpha=0.05, hrs=1,
                        lam_x=2.22, lam_y=2.60, lam_s=2.22, lam_o=2.60, lam_r=math.nan, delta=math.nan,
                        nsim=2000, X=T["X"].data_ptr(), Y=T["Y"].data_ptr(), xy_stride=0,
                        perm=T["perm"].data_ptr(), lap_ni_x=T["lx"].data_ptr(), lap_ni_y=T["ly"].data_ptr(),
                        lap_local=T["ll"].data_ptr(), lap_central=T["lc"].data_ptr(),
                        mix_z=T["mz"].data_ptr(), mix_l=T["ml"].data_ptr())
    ok = C.c_int(-1)
    _lib.check(_lib.lib.dcor_panel_dict_probe(C.c_void_p(T["X"].data_ptr()), C.c_void_p(T["Y"].data_ptr()),
                                              n, C.byref(ok)))
    assert ok.value == (1 if kind in ("coded", "d256") else 0), (kind, ok.value)
    out = torch.empty((R, 6), dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.dcor_premat_subg_launch(C.byref(d), C.c_void_p(out.data_ptr()), None))
    got = out.cpu().numpy()
    # the prepared-panel entry (encoding hoisted out of the launch) gives identical bits
    pn = C.c_void_p()
    _lib.check(_lib.lib.dcor_panel_create(C.c_void_p(T["X"].data_ptr()), C.c_void_p(T["Y"].data_ptr()),
                                          n, None, C.byref(pn)))
    coded = C.c_int(-1)
    _lib.check(_lib.lib.dcor_panel_coded(pn, C.byref(coded)))
    assert coded.value == ok.value
    out2 = torch.full((R, 6), -7.0, dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.dcor_premat_subg_panel_launch(C.byref(d), pn, C.c_void_p(out2.data_ptr()), None))
    _lib.check(_lib.lib.dcor_panel_destroy(pn))
    np.testing.assert_array_equal(out2.cpu().numpy().view(np.int64), got.view(np.int64))
    if kind == "coded" and n == 1003:  # misaligned noise rows are refused, not misread
        d.lap_local = T["ll"].data_ptr() + 4
        assert _lib.lib.dcor_premat_subg_launch(C.byref(d), C.c_void_p(out.data_ptr()), None) == \
            _lib.DCOR_EINVAL
    for r in range(R):
        st, ni, km = orc.ni_subg(age, bmi, eps, eps, hrs=1, lam_x=2.22, lam_y=2.60, perm=perms[r],
                                 lap_x=lx[r], lap_y=ly[r])
        assert list(km) == [k, m]
        st, it, _ = orc.int_subg(age, bmi, eps, eps, hrs=1, lam_s=2.22, lam_o=2.60, lap_local=ll[r],
                                 lap_central=lc[r], mix_z=mz[r], mix_l=ml[r])
        assert_close(got[r], np.concatenate([ni, it]), what=f"hrs {kind} rep {r}")


# ------------------------------------------------------------ edge semantics
def test_k_equals_one_is_na(dc, orc):
    g = np.random.default_rng(3)
    cs = sign_case(g, 200, 0.2, 0.2)
    assert cs["k"] == 1
    got = dc.ci_NI_signbatch(cs["X"], cs["Y"], 0.2, 0.2, noise={"lap_sc": cs["lap_ni_sc"], "lap_x": cs["lap_x"],
                                                                "lap_y": cs["lap_y"]})
    assert math.isfinite(got["rho_hat"]) and np.all(np.isnan(got["ci"]))


def test_nan_tail_only_hits_int(dc, orc):
    """normalise=F: a NaN beyond k*m reaches INT (all n) but not NI (first k*m only)."""
    g = np.random.default_rng(4)
    cs = sign_case(g, 1003, 1.0, 1.0)
    X = cs["X"].copy()
    X[-1] = np.nan
    ni = dc.ci_NI_signbatch(X, cs["Y"], 1.0, 1.0, normalise=False,
                            noise={"lap_sc": cs["lap_ni_sc"], "lap_x": cs["lap_x"], "lap_y": cs["lap_y"]})
    _, ref = orc.ci_ni_signbatch(X, cs["Y"], 1.0, 1.0, 0.05, 0, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
    assert_close([ni["rho_hat"], *ni["ci"]], ref)
    assert math.isfinite(ni["rho_hat"])
    it = dc.ci_INT_signflip(X, cs["Y"], 1.0, 1.0, normalise=False, noise={
        "lap_sc": cs["lap_int_sc"], "flips": cs["flips"], "lap_z": cs["lap_z"], "mix_z": cs["mix_z"],
        "mix_l": cs["mix_l"]})
    assert math.isnan(it["rho_hat"])
    # normalise=T: the NaN reaches the DP mean -> everything NA, as in R
    ni = dc.ci_NI_signbatch(X, cs["Y"], 1.0, 1.0, noise={"lap_sc": cs["lap_ni_sc"], "lap_x": cs["lap_x"],
                                                          "lap_y": cs["lap_y"]})
    assert math.isnan(ni["rho_hat"])


def test_subg_nan_propagates(dc, orc):
    g = np.random.default_rng(5)
    cs = subg_case(g, 1000, 1.0, 1.0)
    X = cs["X"].copy()
    X[17] = np.nan
    got = dc.ci_INT_subG(X, cs["Y"], 1.0, 1.0, noise={"lap_local": cs["lap_local"], "lap_central": cs["lap_central"],
                                                       "mix_z": cs["mix_z"], "mix_l": cs["mix_l"]})
    _, ref, _ = orc.int_subg(X, cs["Y"], 1.0, 1.0, lap_local=cs["lap_local"], lap_central=cs["lap_central"],
                             mix_z=cs["mix_z"], mix_l=cs["mix_l"])
    assert np.all(np.isnan(ref)) and math.isnan(got["rho_hat"])


def test_hrs_sd_zero_branch_gpu(dc):
    n = 50
    got = dc.ci_INT_subG(np.ones(n), np.ones(n), 2.0, 2.0, hrs=True, lambda_sender=3.0, lambda_other=3.0,
                         lambda_receiver=10.0, noise={"lap_local": np.zeros(n), "lap_central": 0.0,
                                                      "mix_z": np.zeros(2000), "mix_l": np.zeros(2000)})
    w = dc.qnorm(0.975) * math.sqrt(2) * (2 * 10.0 / (n * 2.0))
    assert got["rho_hat"] == 1.0 and got["ci"][0] == 1.0 - w and got["ci"][1] == 1.0


def test_errors_mirror_stopifnot(dc):
    with pytest.raises(dc.KLessThanOne):
        dc.ci_NI_signbatch(np.ones(5), np.ones(5), 0.2, 0.2, noise={"lap_sc": np.zeros(4), "lap_x": [], "lap_y": []})
    with pytest.raises(dc.DcorError):
        dc.ci_INT_signflip(np.ones(5), np.ones(4), 1.0, 1.0)
    with pytest.raises(dc.DcorError):
        dc.simulate(dc.CellSpec(n=100, rho=0.5, eps1=-1, eps2=1), 4)


def test_int_only_call_with_n_smaller_than_m(dc, orc):
    """ci_INT_signflip has no batch requirement: n=5 < m=8 must work."""
    g = np.random.default_rng(6)
    cs = sign_case(g, 5, 1.0, 1.0)
    got = dc.ci_INT_signflip(cs["X"], cs["Y"], 1.0, 1.0, noise={
        "lap_sc": cs["lap_int_sc"], "flips": cs["flips"], "lap_z": cs["lap_z"], "mix_z": cs["mix_z"],
        "mix_l": cs["mix_l"]})
    _, ref, _ = orc.ci_int_signflip(cs["X"], cs["Y"], 1.0, 1.0, 0.05, 0, 1, cs["lap_int_sc"], cs["flips"],
                                    cs["lap_z"], cs["mix_z"], cs["mix_l"])
    assert_close([got["rho_hat"], *got["ci"]], ref)


# ----------------------------------------------------------- fused engine
@pytest.mark.parametrize("spec", [
    dict(n=200, rho=0.3, eps1=0.2, eps2=0.2, family="sign", dgp="gaussian"),   # k = 1: NA CIs
    dict(n=5000, rho=-0.5, eps1=0.5, eps2=1.5, family="sign", dgp="bernoulli"),
    dict(n=3000, rho=0.8, eps1=1.0, eps2=1.0, family="subG", dgp="bernoulli"),
    dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", nsim=2000),
    dict(n=999, rho=0.15, eps1=1.5, eps2=0.5, family="sign", dgp="bounded_factor"),
    # mixquant sizes around the wave-select layouts (16 / 32 keys per lane, partial lanes)
    dict(n=1500, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", nsim=1),
    dict(n=1500, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", nsim=7),
    dict(n=1500, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", nsim=1025),
    dict(n=1500, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="bernoulli", nsim=2048),
    dict(n=2500, rho=0.4, eps1=1.0, eps2=1.0, family="subG", dgp="mix_gaussian", nsim=1999),
])
def test_fused_edge_cells(dc, orc, spec):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(seed=77, **spec)
    got = simulate(cell, 12).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 0, 12)
    assert_close(got, ref, what=str(spec))


def test_accumulate_kernel_matches_detail(dc):
    from dcor.sim import CellSpec, accum_from_bytes, accumulate, detail_frame, finalize, simulate
    cell = CellSpec(n=400, rho=0.3, eps1=0.2, eps2=0.2, family="sign", seed=5)  # k=0.. -> n=400,m=200,k=2
    rec = simulate(cell, 3000)
    acc = accum_from_bytes(accumulate(rec, cell.rho).cpu().numpy().tobytes())
    d = detail_frame(rec.cpu().numpy(), cell.rho)
    for a, m in zip(acc, ("ni", "int")):
        hat, lo, up = d[f"{m}_hat"], d[f"{m}_low"], d[f"{m}_up"]
        assert a.n == 3000
        assert a.n_na_est == int(np.isnan(hat).sum())
        assert a.n_cover == int(np.nansum(d[f"{m}_cover"] == 1))
        s = finalize(a, cell.rho)
        assert abs(s["mse"] - np.mean((hat - cell.rho) ** 2)) < 1e-14
        assert abs(s["var"] - np.var(hat, ddof=1)) < 1e-13
        assert abs(s["ci_length"] - np.mean(up - lo)) < 1e-14


def test_headline_full_size_invariants(dc):
    """Full headline size (n = 1e5): CIs ordered and inside [-1,1]; split invariance;
    per-replicate determinism across launches."""
    from dcor.sim import headline_cell, simulate
    cell = headline_cell()
    a = simulate(cell, 1024, 5000).cpu().numpy()
    b = simulate(cell, 1024, 5000).cpu().numpy()
    assert np.array_equal(a, b)
    c = simulate(cell, 512, 5512).cpu().numpy()
    assert np.array_equal(a[512:], c)
    for off in (0, 3):
        lo, hat, hi = a[:, 1 + off], a[:, 0 + off], a[:, 2 + off]
        assert np.all(lo <= hi) and np.all(lo >= -1) and np.all(hi <= 1)
        assert np.all(np.isfinite(hat))
    # INT estimates are sin(.) of the Laplace-noised flip average; NI CIs contain rho most of the time
    cov = np.mean((a[:, 1] <= 0.5) & (0.5 <= a[:, 2]))
    assert 0.9 < cov < 0.99


def test_mc_coverage_vs_independent_restatement(dc):
    """Monte-Carlo coverage of the GPU engine (Philox) vs the numpy restatement driven by
    an independent RNG (numpy PCG64): two-proportion z-test, |z| < 4.5."""
    import numpy_ref as R
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian",
                    mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    B = 20000
    a = simulate(cell, B).cpu().numpy()
    g = np.random.default_rng(99)
    Bn = 1500
    cov_ref = np.zeros((Bn, 2))
    for b in range(Bn):
        cs = sign_case(g, 1000, 1.0, 1.0, rho=0.5)
        ni = R.ci_ni_signbatch(cs["X"], cs["Y"], 1.0, 1.0, 0.05, True, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
        it = R.ci_int_signflip(cs["X"], cs["Y"], 1.0, 1.0, 0.05, 0, True, cs["lap_int_sc"], cs["flips"],
                               cs["lap_z"], cs["mix_z"], cs["mix_l"])
        cov_ref[b] = [ni[1] <= 0.5 <= ni[2], it[1] <= 0.5 <= it[2]]
    for j, off in enumerate((0, 3)):
        p1 = np.mean((a[:, 1 + off] <= 0.5) & (0.5 <= a[:, 2 + off]))
        p2 = cov_ref[:, j].mean()
        p = (p1 * B + p2 * Bn) / (B + Bn)
        z = (p1 - p2) / math.sqrt(p * (1 - p) * (1 / B + 1 / Bn))
        assert abs(z) < 4.5, (j, p1, p2, z)


def test_perm_bitexact_and_valid(dc, orc):
    """dcor_perm_launch (HRS random batches) equals the oracle's restatement and is an
    ordered sample without replacement."""
    import torch
    from dcor import _lib
    n, count, reps = 19433, 19432, 3
    out = torch.empty((reps, count), dtype=torch.int32, device="cuda")
    _lib.check(_lib.lib.dcor_perm_launch(322, _lib.SITE_PERM, 7, reps, n, count,
                                         C.c_void_p(out.data_ptr()), None))
    got = out.cpu().numpy()
    for r in range(reps):
        ref = orc.perm(322, _lib.SITE_PERM, 7 + r, n, count)
        assert np.array_equal(got[r], ref)
        assert len(np.unique(got[r])) == count and got[r].min() >= 0 and got[r].max() < n
