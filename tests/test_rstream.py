"""CPU tests of the R-stream restatement (oracle/dcor_rstream.c).

Pins: values R prints for set.seed + runif / rnorm / rexp and for 2x2 eigen()
(tests/golden/r_known_values.json); AS241 qnorm against scipy's ndtri; exp_rand's table
against its series; the double-double log against correctly rounded values (decimal) and
against glibc's log, which is what R calls.  Draw-order and law checks of whole replicates.
"""
import json
import math
import os
from decimal import Decimal, getcontext

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "r_known_values.json")))


@pytest.fixture(scope="module")
def orc():
    from oracle import oracle
    return oracle


@pytest.mark.parametrize("case", GOLD["streams"], ids=lambda c: f"{c['call']}-{c['seed']}")
def test_r_printed_streams(orc, case):
    kind = {"runif": "unif", "rnorm": "norm", "rexp": "exp"}[case["call"]]
    got = orc.rs_stream(case["seed"], kind, case["n"])
    want = np.array(case["values"])
    # R prints the vector with `decimals` places: agree to half a unit in the last one
    tol = 0.5 * 10.0 ** -case["decimals"] + 1e-15
    assert np.all(np.abs(got - want) <= tol), (got, want)


@pytest.mark.parametrize("case", GOLD["eigen"], ids=lambda c: str(c["abc"]))
def test_r_printed_eigen(orc, case):
    vals, vecs = orc.rs_eigen2(*case["abc"])
    np.testing.assert_allclose(vals, case["values"], rtol=1e-15)
    np.testing.assert_allclose(vecs.T.ravel(), case["vectors"], atol=5e-8)


def test_eigen_sign_convention_matches_r_across_rho(orc):
    """dlaev2's vectors for [[s1^2, s1 s2 rho], [., s2^2]]: (cs, sn) of the larger root first."""
    for rho in (-0.9, -0.3, 0.0, 0.15, 0.5, 0.9):
        for s in ((2.0, 2.0), (1.0, 1.0), (2.0, 0.5)):
            a, b, c = s[0] ** 2, s[0] * s[1] * rho, s[1] ** 2
            v, V = orc.rs_eigen2(a, b, c)
            S = np.array([[a, b], [b, c]])
            assert v[0] >= v[1]
            np.testing.assert_allclose(S @ V, V * v, atol=1e-14)
            np.testing.assert_allclose(V.T @ V, np.eye(2), atol=1e-15)
            A = orc.rs_mvrnorm_factor(np.array(s), rho).reshape(2, 2)
            np.testing.assert_allclose(A @ A.T, S, rtol=1e-14, atol=1e-14)


def test_qnorm5_against_ndtri(orc):
    from scipy.special import ndtri
    g = np.random.default_rng(5)
    ps = np.concatenate([g.uniform(0, 1, 20000), 10.0 ** -g.uniform(1, 18, 5000),
                         1 - 10.0 ** -g.uniform(1, 15, 5000)])
    ps = ps[(ps > 0) & (ps < 1) & (ps != 0.5)]
    got = np.array([orc.lib.orc_rs_qnorm5(float(p)) for p in ps])
    ref = ndtri(ps)
    assert np.max(np.abs(got - ref) / np.abs(ref)) < 3e-15
    assert abs(orc.lib.orc_rs_qnorm5(0.975) - 1.959963984540054) <= 4.5e-16


def test_exp_rand_table_is_the_series(orc):
    import ctypes as C
    getcontext().prec = 60
    q = (C.c_double * 16).in_dll(orc.lib, "orc_rs_exp_q")
    ln2, s, t = Decimal(2).ln(), Decimal(0), Decimal(1)
    for k in range(1, 17):
        t = t * ln2 / k
        s += t
        assert abs(q[k - 1] - float(s)) <= 2.3e-16, k


def test_log_correctly_rounded_and_agrees_with_glibc(orc):
    getcontext().prec = 50
    g = np.random.default_rng(11)
    # the arguments R-stream draws take: 1 - 2|u - 1/2| (Laplace) and min(p, 1-p) (qnorm tails)
    w = g.integers(0, 2 ** 32, 40000, dtype=np.uint64)
    u = -0.5 + w * 2.0 ** -32
    xs = np.concatenate([1 - 2 * np.abs(u[u != 0]), 10.0 ** -g.uniform(1, 19, 4000)])
    cr_miss = glibc_miss = 0
    for x in xs[:8000]:
        cr = float(Decimal(float(x)).ln())
        cr_miss += orc.lib.orc_rs_log(float(x)) != cr
    for x in xs:
        glibc_miss += orc.lib.orc_rs_log(float(x)) != math.log(float(x))
    assert cr_miss == 0
    assert glibc_miss <= 0.005 * len(xs)
    assert orc.lib.orc_rs_log(1.0) == 0.0


def test_rbinom_flip_never_loops(orc):
    """rbinom(1, p) redraws only if u - q >= q * (p/q): impossible for 32-bit uniforms at the
    flip probabilities exp(e)/(exp(e)+1), so the engine's single comparison is R's result."""
    umax = (2 ** 32 - 1) * 2.0 ** -32
    for eps in (0.1, 0.2, 0.5, 1.0, 1.5, 2.0, 5.0, 10.0, 30.0):
        pp = math.exp(eps) / (math.exp(eps) + 1)
        p = min(pp, 1 - pp)
        q = 1 - p
        assert umax - q < q * (p / q)


def _cell(**kw):
    from dcor import CellSpec
    base = dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian",
                mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    base.update(kw)
    return CellSpec(**base).to_c()


def test_replicate_draw_order_and_law(orc):
    c = _cell(n=20000)
    d = orc.rs_draw_reps(c, 2)
    for a in d:
        X, Y = a["X"], a["Y"]
        assert abs(np.corrcoef(X, Y)[0, 1] - 0.5) < 0.03
        assert abs(X.mean() - 0.5) < 0.06 and abs(X.std() - 2.0) < 0.06
        assert a["k"] == 2500 and a["has_mix"] == 1
        assert set(np.unique(a["flips"])) <= {0, 1}
        p = math.e / (math.e + 1)
        assert abs(a["flips"].mean() - p) < 0.02
        assert np.all(np.abs(a["mix_l"]) > 0)
        assert abs(np.mean(a["mix_l"] > 0) - 0.5) < 0.06
    # consecutive replicates continue one stream: the second differs from the first
    assert not np.array_equal(d[0]["X"], d[1]["X"])
    # the first replicate's first normal is R's first rnorm after set.seed
    z1 = orc.rs_stream(1_000_073, "norm", 1)[0]
    A = orc.rs_mvrnorm_factor(np.array([2.0, 2.0]), 0.5)
    zn = orc.rs_stream(1_000_073, "norm", 20001)[20000]
    assert d[0]["X"][0] == 0.5 + ((0.0 + z1 * A[0]) + zn * A[1])


def test_bounded_factor_rho0_draws_nothing_for_u(orc):
    """runif(n, -0, 0) returns -0 without drawing (R's runif: a == b)."""
    c = _cell(family="subG", dgp="bounded_factor", rho=0.0, n=500, mu=(0, 0), sigma=(1, 1))
    d = orc.rs_draw_reps(c, 1)[0]
    e = orc.rs_stream(1_000_073, "word", 1000)
    cE = math.sqrt(3.0)
    e1 = np.array([-cE + (cE - -cE) * orc.lib.orc_rs_word_unif(int(w)) for w in e[:500]])
    np.testing.assert_array_equal(d["X"], -0.0 + e1)


def test_rs_sim_runs_every_family(orc):
    for kw in (dict(), dict(dgp="bernoulli", mu=(0, 0), sigma=(1, 1)),
               dict(family="subG", dgp="bounded_factor", rho=0.3),
               dict(family="subG", dgp="gaussian", mu=(0, 0), sigma=(1, 1)),
               dict(eps1=1.5, eps2=0.5), dict(eps1=0.5, eps2=1.5, normalise=False)):
        out = orc.rs_sim(_cell(**kw), 4)
        assert out.shape == (4, 6) and np.all(np.isfinite(out))
        assert np.all(out[:, 1] <= out[:, 2]) and np.all(out[:, 4] <= out[:, 5])


@pytest.mark.parametrize("case", GOLD["sample"], ids=lambda c: f"sample-{c['seed']}-{c['n']}")
def test_r_printed_sample(orc, case):
    """set.seed(seed); sample(n, size): R_unif_index rejection sampling + do_sample."""
    got = orc.rs_sample_int(case["seed"], case["n"], case["size"]) + 1
    assert list(got) == case["values"]


def test_hrs_run_draws_consume_in_reference_order(orc):
    """run_NI_once: sample.int then rLap(k) x2; run_INT_once: rLap(n), rLap(1), mixquant."""
    n, k, m = 101, 25, 4
    perm, lx, ly = orc.rs_hrs_ni_draws(77, n, k, m)
    assert sorted(perm) == sorted(set(perm)) and len(perm) == k * m
    np.testing.assert_array_equal(perm, orc.rs_sample_int(77, n, k * m))
    ll, lc, mz, ml = orc.rs_hrs_int_draws(78, n, 50)
    w = orc.rs_stream(78, "word", n + 1)
    np.testing.assert_array_equal(ll, [orc.lib.orc_rs_laplace_unit_word(int(x)) for x in w[:n]])
    assert lc == orc.lib.orc_rs_laplace_unit_word(int(w[n]))


def test_mt_words_match_numpy_mt19937(orc):
    """An independent MT19937 (numpy's bit generator) loaded with set.seed's scrambled state
    produces the same tempered words for 2e5 draws."""
    for seed in (1, 1_000_073, 2 ** 31 - 1):
        st = orc.rs_state(seed)
        bg = np.random.MT19937()
        bg.state = {"bit_generator": "MT19937",
                    "state": {"key": np.array(st.mt[:], dtype=np.uint32), "pos": 624}}
        np.testing.assert_array_equal(bg.random_raw(200_000).astype(np.uint32),
                                      orc.rs_stream(seed, "word", 200_000))


def _mt_raw_numpy(st_mt, count):
    """Raw (untempered) MT19937 words: R[0..623] = the state block, then the recurrence
    w[t] = w[t-227] ^ twist(upper(w[t-624]) | lower(w[t-623])), 227 words at a time."""
    R = np.zeros(count, dtype=np.uint32)
    R[:624] = np.array(st_mt[:], dtype=np.uint32)
    t = 624
    while t < count:
        e = min(t + 227, count)
        y = (R[t - 624:e - 624] & np.uint32(0x80000000)) | (R[t - 623:e - 623] & np.uint32(0x7FFFFFFF))
        R[t:e] = R[t - 227:e - 227] ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908B0DF),
                                                                      np.uint32(0))
        t = e
    return R


@pytest.mark.parametrize("seed,J", [(1_000_073, 0), (1_000_073, 1), (7, 20000), (2 ** 31 - 1, 61234)])
def test_mt_jump_ahead_matches_sequential(orc, seed, J):
    """dcor_rstream_mt_jump (host: Berlekamp-Massey characteristic polynomial, x^J mod phi, GF(2)
    combination of raw words) lands on the window the recurrence reaches J words later."""
    import ctypes as C
    from dcor import _lib
    st = orc.rs_state(seed)
    R = _mt_raw_numpy(st.mt, 624 + J + 624)
    out = (C.c_uint32 * 624)()
    assert _lib.lib.dcor_rstream_mt_jump(seed, J, out) == 0, _lib.last_error()
    np.testing.assert_array_equal(np.frombuffer(out, dtype=np.uint32), R[624 + J:624 + J + 624])
