"""GPU tests of the R drop-in surface's .Call routines, run through the stub R runtime
(tests/rstub/) exactly as R would call them: the arithmetic halves of the generators and DP
helpers (whose draws the R wrappers take with R's RNG) against the oracle / a plain restatement
in R's operation order, and the grid routine against the Python grid driver."""
import ctypes as C

import numpy as np
import pytest

from helpers import assert_close
from rstub_py import RStub

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rs():
    import torch
    assert torch.cuda.is_available()
    return RStub()


@pytest.fixture(scope="module")
def orc():
    from oracle import oracle
    return oracle


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.uint64)


@pytest.mark.parametrize("rho", [-1.0, -0.35, 0.0, 0.5, 1.0])
def test_gen_bernoulli(rs, orc, rho):
    g = np.random.default_rng(7)
    n = 4097
    u, v = g.random(n), g.random(n)
    xy = rs.value(rs.call("dcor_R_gen_bernoulli", rs.real(u), rs.real(v), rs.real(rho)))
    X, Y = np.zeros(n), np.zeros(n)
    D = C.POINTER(C.c_double)
    orc.lib.orc_gen_bernoulli(u.ctypes.data_as(D), v.ctypes.data_as(D), n, rho, X.ctypes.data_as(D),
                              Y.ctypes.data_as(D))
    assert xy.shape == (n, 2)
    assert np.array_equal(xy[:, 0], X) and np.array_equal(xy[:, 1], Y)


def test_gen_bernoulli_refuses_rho_beyond_one(rs):
    from rstub_py import RError
    with pytest.raises(RError, match="abs"):
        rs.call("dcor_R_gen_bernoulli", rs.real([0.1]), rs.real([0.2]), rs.real(1.5))


def test_gen_bounded_factor(rs):
    g = np.random.default_rng(8)
    n = 1001
    cU, cE = np.sqrt(3 * 0.4), np.sqrt(3 * 0.6)
    U, E1, E2 = -cU + 2 * cU * g.random(n), -cE + 2 * cE * g.random(n), -cE + 2 * cE * g.random(n)
    xy = rs.value(rs.call("dcor_R_gen_bounded_factor", rs.real(U), rs.real(E1), rs.real(E2)))
    assert np.array_equal(xy[:, 0], U + E1) and np.array_equal(xy[:, 1], U + E2)


def _mvn(z, n, mu, A):
    a, b = z[:n], z[n:]
    return mu[0] + ((0.0 + a * A[0]) + b * A[1]), mu[1] + ((0.0 + a * A[2]) + b * A[3])


@pytest.mark.parametrize("sigma,rho", [((2.0, 2.0), 0.5), ((1.0, 1.0), -0.9), ((2.0, 0.1), -0.95),
                                       ((1.0, 1.0), 0.0), ((3.0, 1.0), 1.0)])
def test_mvrnorm_is_r_arithmetic(rs, orc, sigma, rho):
    """MASS::mvrnorm's transform: LAPACK's eigenvectors (the R-stream restatement pinned to values
    R prints) and dgemm's summation order, bit for bit."""
    g = np.random.default_rng(9)
    n = 777
    z = g.standard_normal(2 * n)
    mu = (0.5, -1.25)
    xy = rs.value(rs.call("dcor_R_mvrnorm", rs.real(z), rs.real(n), rs.real(mu), rs.real(sigma), rs.real(rho)))
    X, Y = _mvn(z, n, mu, orc.rs_mvrnorm_factor(sigma, rho))
    assert np.array_equal(_bits(xy[:, 0]), _bits(X)) and np.array_equal(_bits(xy[:, 1]), _bits(Y))


def test_mix_gaussian(rs, orc):
    g = np.random.default_rng(10)
    n0, n1, rho = 300, 212, 0.6
    z0, z1 = g.standard_normal(2 * n0), g.standard_normal(2 * n1)
    perm = g.permutation(n0 + n1)
    mu0, s0, mu1, s1 = (0.0, 0.0), (1.0, 1.0), (3.0, 3.0), (2.0, 0.5)
    xy = rs.value(rs.call("dcor_R_mix_gaussian", rs.real(z0), rs.real(n0), rs.real(z1), rs.real(n1),
                          rs.integer(perm), rs.real(rho), rs.real(mu0), rs.real(s0), rs.real(mu1), rs.real(s1)))
    X0, Y0 = _mvn(z0, n0, mu0, orc.rs_mvrnorm_factor(s0, rho))
    X1, Y1 = _mvn(z1, n1, mu1, orc.rs_mvrnorm_factor(s1, rho))
    X, Y = np.concatenate([X0, X1])[perm], np.concatenate([Y0, Y1])[perm]
    X, Y = np.clip(X, -1, 1), np.clip(Y, -1, 1)
    assert np.array_equal(_bits(xy[:, 0]), _bits(X)) and np.array_equal(_bits(xy[:, 1]), _bits(Y))


def test_dp_mean_and_standardize(rs, orc):
    g = np.random.default_rng(11)
    x = np.round(g.normal(65, 12, 5000))
    D = C.POINTER(C.c_double)
    got = rs.value(rs.call("dcor_R_dp_mean", rs.real(x), rs.real(45), rs.real(90), rs.real(0.1), rs.real(0.37)))[0]
    ref = orc.lib.orc_dp_mean(x.ctypes.data_as(D), len(x), 45.0, 90.0, 0.1, 0.37)
    assert_close(got, ref)
    z = rs.value(rs.call("dcor_R_standardize_dp", rs.real(x), rs.real(45), rs.real(90), rs.real(64.2),
                         rs.real(11.5), rs.real(1e-8)))
    assert np.array_equal(z, (np.minimum(np.maximum(x, 45), 90) - 64.2) / 11.5)


def test_int_subg_sd_uc_and_the_zero_branch(rs, orc):
    """sd(Uc) for the HRS wrapper's branch test (real-data-sims.R:236-241): against the oracle's
    restatement, and exactly 0 when every clipped product is equal -- where ci_INT_subG takes the
    closed-form width and mixquant draws nothing."""
    g = np.random.default_rng(12)
    n = 3001
    X, Y, ll = g.standard_normal(n), g.standard_normal(n), g.laplace(size=n)
    lam = [2.2, 2.6, 62.8, 1.0 / n]
    sd = rs.value(rs.call("dcor_R_int_subg_sd_uc", rs.real(X), rs.real(Y), rs.real(2.0), rs.real(1.0),
                          rs.real(1.0), rs.real(1.0), rs.real(lam), rs.real(ll)))[0]
    S, O = np.clip(X, -lam[0], lam[0]), np.clip(Y, -lam[1], lam[1])
    Uc = np.clip((S + (2 * lam[0] / 2.0) * ll) * O, -lam[2], lam[2])
    assert_close(sd, orc.r_var(Uc) ** 0.5, rtol=1e-12)
    # Y = 0: every Uc is 0
    Z = np.zeros(n)
    sd0 = rs.value(rs.call("dcor_R_int_subg_sd_uc", rs.real(X), rs.real(Z), rs.real(2.0), rs.real(1.0),
                           rs.real(1.0), rs.real(1.0), rs.real(lam), rs.real(ll)))[0]
    assert sd0 == 0.0
    got = rs.value(rs.call("dcor_R_ci_INT_subG", rs.real(X), rs.real(Z), rs.real(2.0), rs.real(1.0),
                           rs.real(1.0), rs.real(1.0), rs.real(0.05), rs.logical(True), rs.real(lam[0]),
                           rs.real(lam[1]), rs.real(lam[2]), rs.real(lam[3]), rs.real(ll), rs.real(0.3),
                           rs.real([0.0]), rs.real([0.0])))
    st, ref, _ = orc.int_subg(X, Z, 2.0, 1.0, hrs=1, lam_s=lam[0], lam_o=lam[1], lam_r=lam[2],
                              delta=lam[3], lap_local=ll, lap_central=0.3, mix_z=np.zeros(1),
                              mix_l=np.zeros(1))
    assert st == 0
    assert_close(got, ref)


def test_grid_routine_equals_python_grid(rs):
    """dcor_R_grid_run (the .Call behind run_sim_one and dcor_grid) on three cells: the summaries and
    detail records equal dcor.sim.run_grid's."""
    from dcor.sim import CellSpec, run_grid
    cells = [CellSpec(n=2000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_001),
             CellSpec(n=2500, rho=0.3, eps1=1.5, eps2=0.5, family="subG", dgp="bounded_factor", seed=1_000_002),
             CellSpec(n=3000, rho=0.65, eps1=0.5, eps2=0.5, dgp="bernoulli", seed=1_000_003)]
    B = 97
    nc = len(cells)
    col = lambda f: [f(c) for c in cells]  # noqa: E731
    fam = {"sign": 0, "subG": 1}
    dg = {"gaussian": 0, "bernoulli": 1, "bounded_factor": 2, "mix_gaussian": 3}
    out = rs.value(rs.call(
        "dcor_R_grid_run", rs.integer(col(lambda c: fam[c.family])), rs.integer(col(lambda c: dg[c.dgp])),
        rs.real(col(lambda c: c.n)), rs.real(col(lambda c: c.rho)), rs.real(col(lambda c: c.eps1)),
        rs.real(col(lambda c: c.eps2)), rs.real([0.05] * nc), rs.real(col(lambda c: c.mu[0])),
        rs.real(col(lambda c: c.mu[1])), rs.real(col(lambda c: c.sigma[0])), rs.real(col(lambda c: c.sigma[1])),
        rs.logical([True] * nc), rs.integer([0] * nc), rs.real(col(lambda c: c.seed)), rs.real(B),
        rs.logical(True), rs.real([0, 0, 1, 1, 3, 3, 2, 0.5, 0.5]), rs.logical(False),
        rs.real([1000] * nc), rs.integer([0])))
    summ, det = out[:2]
    ref = run_grid(cells, B, detail=True, devices=[0])
    assert np.array_equal(_bits(det.reshape(nc * B, 6)), _bits(np.concatenate([r["records"] for r in ref])))
    for i, r in enumerate(ref):
        for m, meth in enumerate(("NI", "INT")):
            s = summ[(2 * i + m) * 5:(2 * i + m + 1) * 5]
            want = [r["summary"][meth][k] for k in ("mse", "bias", "var", "coverage", "ci_length")]
            assert np.array_equal(_bits(s), _bits(want))


def _grid_call(rs, cells, B, detail=True):
    nc = len(cells)
    col = lambda f: [f(c) for c in cells]  # noqa: E731
    fam = {"sign": 0, "subG": 1}
    dg = {"gaussian": 0, "bernoulli": 1, "bounded_factor": 2, "mix_gaussian": 3}
    return rs.call(
        "dcor_R_grid_run", rs.integer(col(lambda c: fam[c.family])), rs.integer(col(lambda c: dg[c.dgp])),
        rs.real(col(lambda c: c.n)), rs.real(col(lambda c: c.rho)), rs.real(col(lambda c: c.eps1)),
        rs.real(col(lambda c: c.eps2)), rs.real([0.05] * nc), rs.real(col(lambda c: c.mu[0])),
        rs.real(col(lambda c: c.mu[1])), rs.real(col(lambda c: c.sigma[0])), rs.real(col(lambda c: c.sigma[1])),
        rs.logical([True] * nc), rs.integer([0] * nc), rs.real(col(lambda c: c.seed)), rs.real(B),
        rs.logical(detail), rs.real([0, 0, 1, 1, 3, 3, 2, 0.5, 0.5]), rs.logical(False),
        rs.real([1000] * nc), rs.integer([0]))


@pytest.mark.parametrize("family", ["sign", "subG"])
def test_grid_routine_tables_equal_python_tables(rs, family):
    """f2 on the R side: dcor_R_grid_run's detail_all and summ_all (vert-cor.R:556-597;
    ver-cor-subG.R:301-333) equal dcor.tables.grid_detail / grid_summary byte for byte -- the
    family's column order, integer (sign) or logical (sub-G) cover with NA, the setting columns,
    data.table's first-appearance group order with a repeated setting pooled, NI rows then INT."""
    from dcor import tables
    from dcor.sim import expand_grid, run_grid
    from rstub_py import INTSXP, LGLSXP, NA_INTEGER
    kw = (dict(family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)) if family == "sign"
          else dict(family="subG", dgp="bounded_factor"))
    cells = expand_grid([1200, 2500], [0.0, 0.5], [(1.0, 1.0), (0.2, 0.2)], **kw)  # (.2, .2) at 1200: k = 6
    cells.append(cells[1])            # a repeated setting: data.table pools its rows into one group
    B = 23
    out = _grid_call(rs, cells, B)
    det_s, cls = rs.frame(rs.elt(out, 2))
    summ_s, cls2 = rs.frame(rs.elt(out, 3))
    assert cls == ["data.frame"] and cls2 == ["data.frame"]
    assert list(rs.attr(rs.elt(out, 2), "row.names")) == [NA_INTEGER, -B * len(cells)]
    res = run_grid(cells, B, detail=True, devices=[0])
    det_p = tables.grid_detail(cells, res)
    assert list(det_s) == list(det_p) == list(tables.detail_order(family))
    cover_type = INTSXP if family == "sign" else LGLSXP
    for j, name in enumerate(det_s):
        got, want = det_s[name], det_p[name]
        if name.endswith("_cover"):
            assert rs.type(rs.elt(rs.elt(out, 2), j)) == cover_type
            want_i = np.where(np.isnan(want), NA_INTEGER, want).astype(np.int64)
            assert np.array_equal(got.astype(np.int64), want_i), name
        elif name == "repl":
            assert rs.type(rs.elt(rs.elt(out, 2), j)) == INTSXP
            assert np.array_equal(got, want), name
        else:
            assert np.array_equal(_bits(got), _bits(want)), name
    summ_p = tables.grid_summary(cells, res)
    assert len(summ_p) == 2 * (len(cells) - 1)
    assert list(summ_s) == list(tables.SUMMARY_ORDER)
    assert summ_s["method"] == [r["method"] for r in summ_p]
    for name in tables.SUMMARY_ORDER[:-1]:
        assert np.array_equal(_bits(summ_s[name]), _bits([r[name] for r in summ_p])), name
    # k = 6 batches at n = 1200, eps = (.2, .2): finite; the NI summary of the pooled group counts 2B rows
    assert np.all(np.isfinite(summ_s["mse"]))


def test_grid_routine_without_detail_has_summ_all_only(rs):
    from dcor.sim import expand_grid
    cells = expand_grid([1000], [0.3], [(1.0, 1.0)], family="sign", dgp="gaussian")
    out = _grid_call(rs, cells, 5, detail=False)
    assert rs.value(rs.elt(out, 2)) is None
    summ, _ = rs.frame(rs.elt(out, 3))
    assert summ["method"] == ["NI", "INT"] and len(summ["mse"]) == 2


def test_grid_routine_refuses_ragged_cells(rs):
    from rstub_py import RError
    from dcor.sim import expand_grid
    cells = expand_grid([1000, 2000], [0.3], [(1.0, 1.0)], family="sign", dgp="gaussian")
    args = [rs.integer([0, 0]), rs.integer([0, 0]), rs.real([1000, 2000]), rs.real([0.3]),  # rho: 1 value
            rs.real([1, 1]), rs.real([1, 1]), rs.real([0.05] * 2), rs.real([0, 0]), rs.real([0, 0]),
            rs.real([1, 1]), rs.real([1, 1]), rs.logical([True] * 2), rs.integer([0, 0]),
            rs.real([1e6 + 1, 1e6 + 2]), rs.real(5), rs.logical(False), rs.real([0, 0, 1, 1, 3, 3, 2, 0.5, 0.5]),
            rs.logical(False), rs.real([1000] * 2), rs.integer([0])]
    assert len(cells) == 2
    with pytest.raises(RError, match="per-cell"):
        rs.call("dcor_R_grid_run", *args)
