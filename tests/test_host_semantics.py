"""Host-side R semantics that need no GPU: the detail table's cover flag, the HRS eps grid,
argument checks of the HRS driver, and the oracle's refusal of cells R refuses."""
import math

import numpy as np
import pytest


def test_r_cover_three_valued_logic():
    """rho >= lo && rho <= up (vert-cor.R:405): FALSE wins over NA, NA over TRUE."""
    from dcor.sim import r_cover
    nan = float("nan")
    lo = np.array([0.1, nan, nan, 0.6, nan, 0.1, 0.1])
    up = np.array([0.9, 0.9, 0.4, nan, nan, nan, 0.3])
    got = r_cover(0.5, lo, up)
    # TRUE, NA&&TRUE=NA, NA&&FALSE=FALSE, FALSE&&NA=FALSE, NA, TRUE&&NA=NA, TRUE&&FALSE=FALSE
    want = np.array([1.0, nan, 0.0, 0.0, nan, nan, 0.0])
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert np.array_equal(got[~np.isnan(want)], want[~np.isnan(want)])


def test_detail_frame_cover_matches_r_logic():
    from dcor.sim import detail_frame
    nan = float("nan")
    rec = np.array([[0.5, 0.6, nan, 0.5, nan, 0.4],
                    [0.5, 0.1, 0.9, nan, nan, nan]])
    d = detail_frame(rec, 0.5)
    assert d["ni_cover"][0] == 0.0          # 0.5 >= 0.6 is FALSE, whatever up is
    assert d["int_cover"][0] == 0.0         # 0.5 <= 0.4 is FALSE
    assert d["ni_cover"][1] == 1.0 and math.isnan(d["int_cover"][1])


def test_eps_grid_is_r_seq_arithmetic():
    """seq(0.25, 2.5, by = 0.1) is from + (0:n) * by, unrounded (real-data-sims.R:411)."""
    from dcor import hrs
    assert len(hrs.EPS_GRID) == 23
    for i, e in enumerate(hrs.EPS_GRID):
        assert e == 0.25 + i * 0.1
    # the six values that differ from their short decimal by one ulp in R as well
    off = [i for i, e in enumerate(hrs.EPS_GRID) if e != round(e, 10)]
    assert off == [6, 7, 12, 14, 17, 19]
    assert hrs.EPS_GRID[6] == 0.8500000000000001


@pytest.mark.parametrize("R", [200, 7, 1])
def test_sweep_summaries_equal_per_eps_summaries(R):
    """The vectorised sweep summaries equal the per-eps means and type-7 quantiles of
    real-data-sims.R:408-437 (hrs._summ) exactly, NaN rows included."""
    from dcor import hrs
    g = np.random.default_rng(R)
    runs = g.standard_normal((23, R, 6)) * 3
    runs[4, min(3, R - 1), 1] = np.nan
    runs[9, 0, 5] = np.nan
    runs[11, 0, 0] = np.nan
    out = hrs.sweep_summaries(hrs.EPS_GRID, runs)
    for i, (e, r) in enumerate(zip(hrs.EPS_GRID, runs)):
        for want, got in ((hrs._summ("NI", e, r[:, 0], r[:, 1], r[:, 2]), out["ni_mean"][i]),
                          (hrs._summ("INT", e, r[:, 3], r[:, 4], r[:, 5]), out["int_mean"][i])):
            assert want.keys() == got.keys()
            for k, v in want.items():
                assert v == got[k] or (isinstance(v, float) and math.isnan(v) and math.isnan(got[k])), (i, k)


@pytest.mark.parametrize("kw", [dict(rng="R", mode="fused", eps_idx=1),
                                dict(mode="fused", keep_noise=True),
                                dict(rng="mt"), dict(mode="stream"), dict(rng="R")])
def test_hrs_replicates_argument_checks_precede_any_device_work(kw):
    """The checks run before the panel is created (no GPU needed to hit them)."""
    from dcor import hrs
    z = np.zeros(10)
    with pytest.raises(ValueError):
        hrs.hrs_replicates(z, z, 2.0, 2.0, 2.0, 4, **kw)


@pytest.mark.parametrize("kw,ok", [
    (dict(), True), (dict(alpha=1.0), True), (dict(alpha=-0.5), True), (dict(alpha=2.0), False),
    (dict(rho=1.0), True), (dict(rho=1.0 + 1e-9), True), (dict(rho=1.01), False),
    (dict(dgp="bernoulli", rho=1.01), False), (dict(dgp="bounded_factor", rho=-0.3), True),
    (dict(dgp="mix_gaussian", rho=-1.2), False),
])
def test_oracle_cell_check(kw, ok):
    """The oracle refuses exactly the cells R stops on (MASS::mvrnorm's positive-definite
    check with tol 1e-6, gen_bernoulli's stopifnot, alpha >= 2)."""
    import ctypes as C

    from dcor.sim import CellSpec
    from oracle import oracle as orc
    base = dict(n=100, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", seed=3)
    base.update(kw)
    c = CellSpec(**base).to_c()
    st = orc.lib.orc_cell_check(C.cast(C.pointer(c), C.c_void_p))
    assert (st == 0) == ok


def test_fork_guard():
    """A process forked after its parent reached the engine (R's mclapply children) gets
    DCOR_EFORK from every compute entry, before any HIP call; the parent keeps working."""
    import ctypes as C
    import os

    import torch
    if torch.cuda.is_available():
        pytest.skip("fork is only exercised on a host without a GPU")
    from dcor import _lib
    z = np.zeros(4)
    P = C.POINTER(C.c_double)
    out = C.c_double()
    st = _lib.lib.dcor_mixquant(z.ctypes.data_as(P), z.ctypes.data_as(P), 4, 1.0, 0.5, C.byref(out))
    assert st == _lib.DCOR_ENODEV          # the parent now owns the engine
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        code = _lib.lib.dcor_mixquant(z.ctypes.data_as(P), z.ctypes.data_as(P), 4, 1.0, 0.5, C.byref(out))
        os.write(w, bytes([code]) + _lib.last_error().encode()[:200])
        os._exit(0)
    os.close(w)
    msg = os.read(r, 256)
    os.waitpid(pid, 0)
    assert msg[0] == _lib.DCOR_EFORK, msg
    assert b"fork" in msg
    st = _lib.lib.dcor_mixquant(z.ctypes.data_as(P), z.ctypes.data_as(P), 4, 1.0, 0.5, C.byref(out))
    assert st == _lib.DCOR_ENODEV
