"""BASELINE config C4 under -m gpu: the full paper sweep of vert-cor.R:19-40 crossed with both
estimator families -- {sign: gaussian, bernoulli; sub-G: gaussian (mu = 0,
sigma = 1), bounded factor} x rho {0, .3, .8} x 5 eps pairs x n {200, 400, 800, 1600, 3200, 1e4,
1e5, 1e6} = 480 cells -- through the batched grid (dcor.sim.run_grid, one dcor_grid_run_multi
call) and compared with the CPU oracle fed the same Philox streams.

Includes the k = 1 cells (n = 200, eps = (.2, .2): m = ceil(8 / .04) = 200, vert-cor.R:207-209;
ver-cor-subG.R:37-38), whose NI sd, CI and cover are NA (sd of one value): the records must be
NaN where the oracle's are, and the accumulators must count them (n_na_ci, n_cover_na)."""
import numpy as np
import pytest

from helpers import assert_close

pytestmark = pytest.mark.gpu

N_GRID = (200, 400, 800, 1600, 3200, 10_000, 100_000, 1_000_000)
B_SMALL = 8      # replicates per cell for n <= 1e5 (every replicate checked for n <= 1e4)
B_LARGE = 2      # replicates per cell at n = 1e6


@pytest.fixture(scope="module")
def c4():
    import torch
    assert torch.cuda.is_available()
    from dcor.sim import paper_grid, run_grid
    cells = paper_grid(n_grid=N_GRID)
    assert len(cells) == 480
    small = [c for c in cells if c.n < 1_000_000]
    large = [c for c in cells if c.n == 1_000_000]
    rs = run_grid(small, B_SMALL, detail=True, devices=[0])
    rl = run_grid(large, B_LARGE, detail=True, devices=[0])
    res = {id(c): r for c, r in zip(small, rs)}
    res.update({id(c): r for c, r in zip(large, rl)})
    return cells, res


def _oracle(cell, r0, r1):
    from oracle.oracle import sim_reps
    return sim_reps(cell.to_c(), r0, r1, threads=8)


def _cover(rho, lo, hi):
    """R's rho >= lo && rho <= hi with NA (1, 0, or NaN)."""
    from dcor.sim import r_cover
    return r_cover(rho, lo, hi)


def test_c4_grid_shape(c4):
    cells, _ = c4
    fam = {(c.family, c.dgp) for c in cells}
    assert fam == {("sign", "gaussian"), ("sign", "bernoulli"), ("subG", "gaussian"), ("subG", "bounded_factor")}
    assert sorted({c.n for c in cells}) == list(N_GRID)
    assert len({c.seed for c in cells}) == 120   # seed 1e6 + i per expand.grid row, per family block


@pytest.mark.parametrize("n", N_GRID)
def test_c4_records_vs_oracle(c4, n):
    """Replicates of every cell of this n against the oracle: all of them for n <= 1e4, the first
    and the last for n = 1e5 and 1e6 (estimates and CI endpoints within 1e-12, NaN where the
    oracle has NaN)."""
    cells, res = c4
    for c in (c for c in cells if c.n == n):
        rec = res[id(c)]["records"]
        B = rec.shape[0]
        picks = range(B) if n <= 10_000 else sorted({0, B - 1})
        for r in picks:
            ref = _oracle(c, r, r + 1)[0]
            assert np.array_equal(np.isnan(rec[r]), np.isnan(ref)), (c, r, rec[r], ref)
            assert_close(rec[r], ref, what=f"C4 cell {c} rep {r}")


def test_c4_k1_cells_are_na(c4):
    """n = 200, eps = (.2, .2): k = 1, so sd(T) is NA and the NI CI and cover are NA; the INT side
    is finite.  Both families, every rho and DGP: 12 cells."""
    cells, res = c4
    k1 = [c for c in cells if c.n == 200 and c.eps1 == 0.2 and c.eps2 == 0.2]
    assert len(k1) == 12
    for c in k1:
        r = res[id(c)]
        rec = r["records"]
        assert np.all(np.isfinite(rec[:, 0]))                          # the NI point estimate exists
        assert np.all(np.isnan(rec[:, 1])) and np.all(np.isnan(rec[:, 2]))
        assert np.all(np.isfinite(rec[:, 3:]))
        ni, it = r["accum"]
        B = rec.shape[0]
        assert (ni.n, ni.n_na_ci, ni.n_cover_na, ni.n_cover, ni.n_na_est) == (B, B, B, 0, 0)
        assert it.n_na_ci == 0 and it.n_cover_na == 0
        s = r["summary"]["NI"]
        assert np.isnan(s["coverage"]) and np.isnan(s["ci_length"]) and np.isfinite(s["mse"])


def test_c4_accumulator_counts_vs_oracle(c4):
    """For every cell with n <= 1e4 (all replicates checked): the accumulators' counts -- n, cover,
    NA cover, NA CI, NA estimate -- equal the counts of the oracle's records."""
    cells, res = c4
    for c in (c for c in cells if c.n <= 10_000):
        r = res[id(c)]
        ref = _oracle(c, 0, r["records"].shape[0])
        for m, acc in enumerate(r["accum"]):
            est, lo, hi = ref[:, 3 * m], ref[:, 3 * m + 1], ref[:, 3 * m + 2]
            cov = _cover(c.rho, lo, hi)
            want = (len(est), int(np.nansum(cov == 1.0)), int(np.isnan(cov).sum()),
                    int((np.isnan(lo) | np.isnan(hi)).sum()), int(np.isnan(est).sum()))
            got = (acc.n, acc.n_cover, acc.n_cover_na, acc.n_na_ci, acc.n_na_est)
            assert got == want, (c, m, got, want)


def test_c4_one_launch_over_all_cells(c4):
    """The 480-cell mixed-family plan in ONE dcor_grid_launch (every kernel family and DGP, n from
    200 to 1e6, per-cell replicate counts): records byte-identical to the two run_grid calls."""
    from dcor.sim import grid_launch
    cells, res = c4
    counts = [B_LARGE if c.n == 1_000_000 else B_SMALL for c in cells]
    out, _ = grid_launch(cells, 0, counts)
    got = out.cpu().numpy()
    ref = np.concatenate([res[id(c)]["records"] for c in cells])
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
