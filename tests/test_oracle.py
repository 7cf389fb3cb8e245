"""CPU tests of the oracle: published known-answer vectors, closed-form KATs from the
reference formulas, R-semantics checks, and agreement with the independent numpy
restatement (tests/numpy_ref.py) and the committed golden fixtures."""
import math
import os

import numpy as np
import pytest

import numpy_ref as R
from helpers import assert_close, sign_case, subg_case, unit_laplace
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "explicit_cases.npz")


# ------------------------------------------------------- published KAT vectors
# Random123 philox4x32_10 known-answer vectors (kat_vectors in the Random123 distribution).
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_kat(ctr, key, want):
    assert tuple(int(v) for v in O.philox(ctr, *key)) == want


def test_u53_open_interval_and_exact():
    assert O.lib.orc_u53(0, 0) == 2.0 ** -53
    assert O.lib.orc_u53(0xffffffff, 0xffffffff) == 1 - 2.0 ** -53
    assert O.lib.orc_u53(0x80000000, 0) == 0.5 + 2.0 ** -53


def test_log_accuracy():
    g = np.random.default_rng(1)
    x = np.concatenate([g.uniform(0, 1, 20000), 2.0 ** -g.uniform(0, 53, 2000), [2 ** -53, 1 - 2 ** -53, 0.5, 1.0]])
    got = np.array([O.lib.orc_log(float(v)) for v in x])
    ref = np.log(x)
    ulp = np.spacing(np.abs(ref)) + (ref == 0)
    assert np.max(np.abs(got - ref) / ulp) <= 2.0


def test_sincospi_accuracy():
    g = np.random.default_rng(2)
    t = 2 * (2 * np.floor(g.uniform(0, 2 ** 52, 20000)) + 1) * 2.0 ** -53
    s = np.zeros(1)
    c = np.zeros(1)
    errs = []
    for v in t:
        O.lib.orc_sincospi(float(v) * 64.0, s.ctypes.data_as(O._D), c.ctypes.data_as(O._D))  # takes 64 t
        errs.append(max(abs(s[0] - math.sin(math.pi * v)), abs(c[0] - math.cos(math.pi * v))))
    assert max(errs) < 1e-15


def test_normal_and_laplace_moments():
    z = O.gen_normals(1234, 0, 6, 400_000)
    assert abs(z.mean()) < 5 * 1 / math.sqrt(len(z))
    assert abs(z.var() - 1) < 0.01
    assert abs(np.mean(z ** 4) - 3) < 0.05
    lap = O.gen_laplace(1234, 0, 7, 400_000)
    assert abs(lap.mean()) < 0.01 and abs(lap.var() - 2) < 0.03
    assert abs(np.mean(np.abs(lap)) - 1) < 0.01


def test_streams_distinct_per_rep_and_site():
    a = O.gen_normals(7, 0, 6, 64)
    assert not np.array_equal(a, O.gen_normals(7, 1, 6, 64))
    assert not np.array_equal(a, O.gen_normals(7, 0, 5, 64))
    assert not np.array_equal(a, O.gen_normals(8, 0, 6, 64))
    assert np.array_equal(a, O.gen_normals(7, 0, 6, 64))


# ----------------------------------------------------------- closed-form KATs
def test_qnorm():
    assert abs(O.qnorm(0.975) - 1.959963984540054) <= 4.5e-16  # R's AS241 double (2 ulp of the true quantile)
    from scipy.special import ndtri
    for p in (1e-10, 0.001, 0.025, 0.3, 0.5, 0.8, 0.995, 1 - 1e-9):
        assert abs(O.qnorm(p) - ndtri(p)) <= 4e-15 * max(1.0, abs(ndtri(p)))


def test_lambda_n_kat():
    # ver-cor-subG.R:1: min(2*sqrt(log n), 2*sqrt(3)) = 2*sqrt(3) for all n >= 21
    for n in (21, 200, 1000, 1e5, 1e6):
        assert O.lambda_n(n) == 2 * math.sqrt(3) == 3.4641016151377544
    assert O.lambda_n(10) == 2 * math.sqrt(math.log(10))
    assert O.lambda_n(20) < 2 * math.sqrt(3)


def test_lambda_int_n_kat():
    # lambda_r = 5*max(eta_r,1)*min(log n, 6)/min(eps_s, 1): 30 (eps_s>=1) or 60 (eps_s=.5), n>=404
    for n in (404, 1e4, 1e5, 1e6):
        assert list(O.lambda_int_n(n, 1, 1, 1.0)) == [2 * math.sqrt(3), 30.0]
        assert list(O.lambda_int_n(n, 1, 1, 1.5)) == [2 * math.sqrt(3), 30.0]
        assert list(O.lambda_int_n(n, 1, 1, 0.5)) == [2 * math.sqrt(3), 60.0]


@pytest.mark.parametrize("eps,m", [((0.2, 0.2), 200), ((0.5, 0.5), 32), ((1.0, 1.0), 8),
                                   ((1.5, 0.5), 11), ((0.5, 1.5), 11)])
def test_batch_size_kat(eps, m):
    assert math.ceil(8 / (eps[0] * eps[1])) == m  # incl. 8/(0.2*0.2) = 199.99999999999997 -> 200


def test_mixquant_index_kat():
    assert math.ceil(0.975 * 1000) == 975 and math.ceil((1 - 0.05 / 2) * 2000) == 1950
    z = np.arange(1000, dtype=float)[::-1].copy()
    assert O.mixquant(z, np.zeros(1000), 0.0, 0.975) == 974.0


def test_mean_of_signs_is_exact_quotient():
    """R's mean() of a batch of signs vs the GPU's integer count / m.  For every batch size
    the configs use (m = 8, 32, 11, 200) it is the correctly rounded c/m for every c and any
    element order (the GPU path is R-exact there); for other m, R's long-double mean can
    double-round (e.g. -11/199) -- at most 1 ulp, far inside the 1e-12 bound."""
    g = np.random.default_rng(0)
    for m in list(range(1, 65)) + [99, 128, 199, 200, 201]:
        for c in range(-m, m + 1):
            v = np.array([1.0] * ((m + c) // 2) + [-1.0] * ((m - c) // 2) + [0.0] * ((m + c) % 2))
            assert len(v) == m and v.sum() == c
            for _ in range(4 if m in (8, 11, 32, 200) else 1):
                g.shuffle(v)
                r = O.r_mean(v)
                if m in (8, 11, 32, 200):
                    assert r == c / m
                else:
                    assert abs(r - c / m) <= np.spacing(abs(c / m))


def test_r_mean_correction_pass():
    x = np.array([1e16, 1.0, -1e16, 3.0])
    assert O.r_mean(x) == R.r_mean(x)
    assert O.r_var(np.array([1.0])) != O.r_var(np.array([1.0]))  # NA


def test_ni_subg_constant_kat():
    # X=Y=c (|c|<lambda), zero noise: xbar=c, rho=(m/k)*k*c^2 = m c^2; sd(T)=0 -> CI=[rho,rho]
    n, c = 80, 0.25
    st, out, km = O.ni_subg(np.full(n, c), np.full(n, c), 1.0, 1.0, lap_x=np.zeros(10), lap_y=np.zeros(10))
    assert st == 0 and list(km) == [10, 8]
    assert out[0] == 8 * c * c and out[1] == out[0] and out[2] == out[0]


def test_ni_sign_kat():
    # normalise=F, X=Y=+1: batch sign means 1, T=m, eta=m, sd(T)=0 (vert-cor.R:233-254)
    n = 40
    st, out = O.ci_ni_signbatch(np.ones(n), np.ones(n), 1.0, 1.0, 0.05, 0, np.zeros(4), np.zeros(5), np.zeros(5))
    assert st == 0
    assert out[0] == math.sin(math.pi * 8.0 / 2) and out[2] == 1.0 and out[1] == math.sin(math.pi * 8.0 / 2)
    st, _ = O.ci_ni_signbatch(np.ones(5), np.ones(5), 1.0, 1.0, 0.05, 0, np.zeros(4), np.zeros(1), np.zeros(1))
    assert st == 2  # k < 1: stopifnot(k >= 1)


def test_ni_sign_k1_is_na():
    # eps=(0.2,0.2), n=200 -> m=200, k=1: sd of one batch product is NA
    g = np.random.default_rng(3)
    st, out = O.ci_ni_signbatch(g.normal(size=200), g.normal(size=200), 0.2, 0.2, 0.05, 1,
                                unit_laplace(g, 4), unit_laplace(g, 1), unit_laplace(g, 1))
    assert st == 0 and np.isfinite(out[0]) and np.isnan(out[1]) and np.isnan(out[2])


def test_int_subg_hrs_sd_zero_branch():
    # real-data-sims.R:237-238: U constant -> sd(Uc)=0 -> width = qnorm*sqrt(2)*(2 lr/(n eps_r))
    n = 50
    st, out, lam = O.int_subg(np.ones(n), np.ones(n), 2.0, 2.0, hrs=1, lam_s=3.0, lam_o=3.0, lam_r=10.0,
                              lap_local=np.zeros(n), lap_central=0.0, mix_z=np.zeros(2000), mix_l=np.zeros(2000))
    w = O.qnorm(0.975) * math.sqrt(2) * (2 * 10.0 / (n * 2.0))
    assert st == 0 and out[0] == 1.0 and out[1] == max(1.0 - w, -1) and out[2] == 1.0


def test_subg_m_gt_n_guard():
    # ver-cor-subG.R:37: if (m > n) m <- n  -> k = 1
    st, out, km = O.ni_subg(np.arange(5.0) / 10, np.arange(5.0) / 10, 0.2, 0.2, lap_x=np.zeros(1), lap_y=np.zeros(1))
    assert st == 0 and list(km) == [1, 5] and np.isnan(out[1])


def test_hrs_k_lt_2_guard():
    # real-data-sims.R:130: if (k < 2) { k <- 2; m <- floor(n/k) }
    n = 9
    perm = np.arange(8, dtype=np.int32)
    st, out, km = O.ni_subg(np.linspace(-1, 1, n), np.linspace(-1, 1, n), 0.5, 0.5, hrs=1, perm=perm,
                            lap_x=np.zeros(2), lap_y=np.zeros(2))
    assert st == 0 and list(km) == [2, 4]


# ------------------------------------------- oracle vs independent restatement
@pytest.mark.parametrize("n", [10, 400, 3000])
@pytest.mark.parametrize("eps", [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5), (0.5, 1.5)])
def test_oracle_vs_numpy_sign(n, eps):
    g = np.random.default_rng(n + int(10 * eps[0]) * 100 + int(10 * eps[1]))
    cs = sign_case(g, n, *eps)
    st, ni = O.ci_ni_signbatch(cs["X"], cs["Y"], *eps, 0.05, 1, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
    ref = R.ci_ni_signbatch(cs["X"], cs["Y"], *eps, 0.05, True, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
    if ref is None:
        assert st == 2
    else:
        assert_close(ni, ref, 1e-13, 1e-14, "NI")
    for mode in (0, 1, 2):
        st, it, _ = O.ci_int_signflip(cs["X"], cs["Y"], *eps, 0.05, mode, 1, cs["lap_int_sc"], cs["flips"],
                                      cs["lap_z"], cs["mix_z"], cs["mix_l"])
        ref = R.ci_int_signflip(cs["X"], cs["Y"], *eps, 0.05, mode, True, cs["lap_int_sc"], cs["flips"],
                                cs["lap_z"], cs["mix_z"], cs["mix_l"])
        assert_close(it, ref, 1e-13, 1e-14, f"INT mode {mode}")


@pytest.mark.parametrize("n", [10, 400, 3000])
@pytest.mark.parametrize("eps", [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5), (0.2, 0.2)])
@pytest.mark.parametrize("hrs", [False, True])
def test_oracle_vs_numpy_subg(n, eps, hrs):
    g = np.random.default_rng(7 * n + int(10 * eps[0]) + 31 * hrs)
    cs = subg_case(g, n, *eps, nsim=2000 if hrs else 1000, hrs=hrs)
    lam = (2.2, 2.6) if hrs else (None, None)
    st, ni, _ = O.ni_subg(cs["X"], cs["Y"], *eps, hrs=int(hrs), lam_x=lam[0] or np.nan, lam_y=lam[1] or np.nan,
                          perm=cs["perm"], lap_x=cs["lap_x"], lap_y=cs["lap_y"])
    ref = R.ni_subg(cs["X"], cs["Y"], *eps, hrs=hrs, lam_x=lam[0], lam_y=lam[1], perm=cs["perm"],
                    lap_x=cs["lap_x"], lap_y=cs["lap_y"])
    assert st == 0
    assert_close(ni, ref, 1e-13, 1e-14, "NI subG")
    st, it, _ = O.int_subg(cs["X"], cs["Y"], *eps, hrs=int(hrs), lam_s=lam[0] or np.nan, lam_o=lam[1] or np.nan,
                           lap_local=cs["lap_local"], lap_central=cs["lap_central"], mix_z=cs["mix_z"],
                           mix_l=cs["mix_l"])
    ref = R.int_subg(cs["X"], cs["Y"], *eps, hrs=hrs, lam_s=lam[0], lam_o=lam[1], lap_local=cs["lap_local"],
                     lap_central=cs["lap_central"], mix_z=cs["mix_z"], mix_l=cs["mix_l"])
    assert st == 0
    assert_close(it, ref, 1e-13, 1e-14, "INT subG")


def test_mvrnorm_factor():
    A = np.zeros(4)
    O.lib.orc_mvrnorm_factor(np.array([0.5, 0.5]).ctypes.data_as(O._D), np.array([2.0, 2.0]).ctypes.data_as(O._D),
                             0.5, A.ctypes.data_as(O._D))
    A = A.reshape(2, 2)
    assert np.allclose(A @ A.T, [[4, 2], [2, 4]], rtol=0, atol=1e-14)
    # R: eigen(matrix(c(1,.5,.5,1),2))$vectors = [[.707,-.707],[.707,.707]]
    assert A[0, 0] > 0 and A[1, 0] > 0 and A[0, 1] < 0 and A[1, 1] > 0


# -------------------------------------------------------------- golden files
def _gold():
    return np.load(GOLD, allow_pickle=False)


def test_golden_oracle():
    d = _gold()
    for i in range(int(d["n_sign"][0])):
        p = f"sign{i}_"
        n, e1, e2, lz = d[p + "scalars"]
        st, ni = O.ci_ni_signbatch(d[p + "X"], d[p + "Y"], e1, e2, 0.05, 1, d[p + "lap_ni_sc"],
                                   d[p + "lap_x"], d[p + "lap_y"])
        if st == 0:
            assert_close(ni, d[p + "ni"], 1e-13, 1e-14, p + "ni")
        else:
            assert np.all(np.isnan(d[p + "ni"]))
        for md in range(3):
            st, it, _ = O.ci_int_signflip(d[p + "X"], d[p + "Y"], e1, e2, 0.05, md, 1, d[p + "lap_int_sc"],
                                          d[p + "flips"], lz, d[p + "mix_z"], d[p + "mix_l"])
            assert_close(it, d[p + "int"][md], 1e-13, 1e-14, p + f"int{md}")
    for i in range(int(d["n_subg"][0])):
        p = f"subg{i}_"
        n, e1, e2, lc, hrs, lx, ly = d[p + "scalars"]
        perm = d[p + "perm"] if hrs else None
        st, ni, _ = O.ni_subg(d[p + "X"], d[p + "Y"], e1, e2, hrs=int(hrs), lam_x=lx, lam_y=ly, perm=perm,
                              lap_x=d[p + "lap_x"], lap_y=d[p + "lap_y"])
        assert_close(ni, d[p + "ni"], 1e-13, 1e-14, p + "ni")
        st, it, _ = O.int_subg(d[p + "X"], d[p + "Y"], e1, e2, hrs=int(hrs), lam_s=lx, lam_o=ly,
                               lap_local=d[p + "lap_local"], lap_central=lc, mix_z=d[p + "mix_z"],
                               mix_l=d[p + "mix_l"])
        assert_close(it, d[p + "int"], 1e-13, 1e-14, p + "int")
    for j in range(12):
        c, want = d[f"mq{j}_c"]
        got = O.mixquant(d[f"mq{j}_z"], d[f"mq{j}_l"], c, 0.975)
        assert got == want or (np.isnan(got) and np.isnan(want))
    for j in range(6):
        eps, L = d[f"ps{j}_par"]
        assert_close(O.priv_standardize(d[f"ps{j}_v"], eps, L, d[f"ps{j}_lap"]), d[f"ps{j}_out"], 1e-13, 1e-14)
        assert_close(O.dp_sd(d[f"sd{j}_x"], 45.0, 90.0, 0.1, 0.1, d[f"sd{j}_lap"]), d[f"sd{j}_out"], 1e-13, 1e-14)


# --------------------------------------------------------- fused restatement
def test_fused_oracle_statistics():
    """Oracle MC coverage of the sign family at a small cell is near nominal."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "distributed-correlation_amd"))
    from dcor.sim import CellSpec
    cell = CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    out = O.sim_reps(cell.to_c(), 0, 400, threads=4)
    cov_ni = np.mean((out[:, 1] <= 0.5) & (0.5 <= out[:, 2]))
    cov_int = np.mean((out[:, 4] <= 0.5) & (0.5 <= out[:, 5]))
    assert 0.85 < cov_ni <= 1.0 and 0.85 < cov_int <= 1.0
    assert abs(np.mean(out[:, 0]) - 0.5) < 0.1 and abs(np.mean(out[:, 3]) - 0.5) < 0.1


def test_mix_gaussian_dgp_law():
    """gen_mix_gaussian (ver-cor-subG.R:113-133) in the oracle's draw streams: the label rate,
    the clipped marginal means and the clip masses match the mixture's closed forms."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "distributed-correlation_amd"))
    from scipy import stats
    from dcor.sim import CellSpec
    n = 400_000
    for pi, mu1, s1 in ((0.5, (3.0, 3.0), (2.0, 0.5)), (0.3, (0.5, -0.5), (0.7, 1.3))):
        cell = CellSpec(n=n, rho=0.4, eps1=1.0, eps2=1.0, family="subG", dgp="mix_gaussian", pi_mix=pi,
                        mix_mu1=mu1, mix_sigma1=s1, seed=99)
        X, Y = O.gen_xy(cell.to_c(), 7)
        assert X.min() >= -1.0 and X.max() <= 1.0 and Y.min() >= -1.0 and Y.max() <= 1.0
        for v, j in ((X, 0), (Y, 1)):
            comps = [(1 - pi, 0.0, 1.0), (pi, mu1[j], s1[j])]
            def clipped_mean(m, s):   # E[clip(N(m, s^2), -1, 1)]
                a, b = (-1 - m) / s, (1 - m) / s
                return (-stats.norm.cdf(a) + stats.norm.sf(b)
                        + m * (stats.norm.cdf(b) - stats.norm.cdf(a)) - s * (stats.norm.pdf(b) - stats.norm.pdf(a)))
            mean = sum(w * clipped_mean(m, s) for w, m, s in comps)
            top = sum(w * stats.norm.sf((1 - m) / s) for w, m, s in comps)
            assert abs(v.mean() - mean) < 5e-3, (pi, j, v.mean(), mean)
            assert abs(np.mean(v == 1.0) - top) < 4e-3, (pi, j)


def test_perm_uniformity():
    """The keyed Feistel permutation (HRS random batches, the role of sample.int): P_r(0)
    and P_r(1) over many replicate keys are uniform and independent enough (chi-square)."""
    from scipy import stats
    n, R = 97, 30_000
    first = np.array([O.perm(11, 8, r, n, 2) for r in range(R)])
    for col in (0, 1):
        cnt = np.bincount(first[:, col], minlength=n)
        assert stats.chisquare(cnt).pvalue > 1e-4, col
    assert np.all(first[:, 0] != first[:, 1])
    # joint residues mod 8 against uniformly random ordered pairs of distinct elements
    pair = np.bincount((first[:, 0] % 8) * 8 + first[:, 1] % 8, minlength=64)
    c = np.bincount(np.arange(n) % 8, minlength=8).astype(float)
    exp = (np.outer(c, c) - np.diag(c)).ravel() / (n * (n - 1)) * R
    assert stats.chisquare(pair, exp).pvalue > 1e-4


def test_gaussian_dgp_law_ziggurat():
    """The Gaussian DGP's draw contract (one DGP_A block per sample, two 1024-layer ziggurat
    normals): MASS::mvrnorm's moments (vert-cor.R:389-394), normal quantiles of the standardised
    marginals, independence of neighbouring samples, and the tail beyond the base layer's
    r = 4.039 drawn at its normal rate."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "distributed-correlation_amd"))
    from scipy import stats
    from dcor.sim import CellSpec
    n = 400_000
    cell = CellSpec(n=n, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, -0.25), sigma=(2.0, 0.5), seed=1234)
    X, Y = O.gen_xy(cell.to_c(), 3)
    zx, zy = (X - 0.5) / 2.0, (Y + 0.25) / 0.5
    se = 1 / math.sqrt(n)
    assert abs(zx.mean()) < 5 * se and abs(zy.mean()) < 5 * se
    assert abs(zx.var() - 1) < 5 * math.sqrt(2) * se and abs(zy.var() - 1) < 5 * math.sqrt(2) * se
    assert abs(np.corrcoef(zx, zy)[0, 1] - 0.5) < 5 * 0.75 * se
    assert stats.kstest(zx, "norm").pvalue > 1e-4 and stats.kstest(zy, "norm").pvalue > 1e-4
    # neighbouring samples (neighbouring Philox counters) are uncorrelated, in both coordinates
    assert abs(np.corrcoef(zx[0::2], zx[1::2])[0, 1]) < 5 * math.sqrt(2) * se
    assert abs(np.corrcoef(zy[0::2], zx[1::2])[0, 1]) < 5 * math.sqrt(2) * se
    # whitened pair (zx and the Cholesky residual of zy): independent N(0, 1); tails near and past
    # the base layer's r occur at 2 (1 - Phi(t)) per coordinate
    z1 = zx
    z2 = (zy - 0.5 * zx) / math.sqrt(0.75)
    assert abs(np.corrcoef(z1, z2)[0, 1]) < 5 * se
    assert stats.kstest(z2, "norm").pvalue > 1e-4
    r = 4.038849846109504
    for z in (z1, z2):
        # |z| > 3.3: 2 (1 - Phi(3.3)) = 9.67e-4 (strips and wedges near the base); > r: the tail
        for t in (3.3, 3.8, r):
            p = 2 * stats.norm.sf(t)
            cnt = int(np.sum(np.abs(z) > t))
            assert abs(cnt - n * p) < 5 * math.sqrt(n * p) + 1, (t, cnt, n * p)
