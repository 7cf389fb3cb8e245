"""Randomised GPU-vs-oracle sweep over the cell space (both families, every DGP, both RNG
modes): small and ragged n, rho at and near +-1, eps from 0.1 to 5, normalise on/off, every
ci_mode.  Bar as elsewhere: 1e-12 relative (1e-13 absolute floor); a status the oracle
returns (k < 1) must be the status the engine returns."""
import numpy as np
import pytest

from helpers import close

pytestmark = pytest.mark.gpu

DGPS = ("gaussian", "bernoulli", "bounded_factor", "mix_gaussian")


def _cells(seed, count):
    from dcor import CellSpec
    g = np.random.default_rng(seed)
    out = []
    for i in range(count):
        fam = "sign" if g.random() < 0.5 else "subG"
        dgp = DGPS[g.integers(0, 4)]
        rho = float(g.choice([-1.0, -0.999, 1.0, 0.0, g.uniform(-1, 1)]))
        if dgp == "bounded_factor":
            rho = abs(rho)
        n = int(g.choice([2, 3, 7, 31, 64, 65, 100, 257, 1000, 4099]))
        e1, e2 = float(np.exp(g.uniform(np.log(0.1), np.log(5)))), float(np.exp(g.uniform(np.log(0.1), np.log(5))))
        out.append(CellSpec(n=n, rho=rho, eps1=e1, eps2=e2, family=fam, dgp=dgp,
                            mu=(float(g.normal()), float(g.normal())),
                            sigma=(float(g.uniform(0.5, 3)), float(g.uniform(0.5, 3))),
                            normalise=bool(g.random() < 0.8),
                            ci_mode=str(g.choice(["auto", "normal", "laplace"])),
                            seed=int(g.integers(1, 2 ** 31 - 1))))
    return out


def _agree(got, ref):
    return close(got, ref, 1e-12, 1e-13)


@pytest.mark.parametrize("block", range(4))
def test_fused_engine_fuzz(block):
    from dcor import _lib
    from dcor.sim import simulate
    from oracle import oracle as orc
    for cell in _cells(100 + block, 12):
        try:
            ref = orc.sim_reps(cell.to_c(), 5, 8)
        except RuntimeError as e:
            with pytest.raises(_lib.DcorError):
                simulate(cell, 3, 5).cpu()
            continue
        got = simulate(cell, 3, 5).cpu().numpy()
        assert _agree(got, ref), (cell, got, ref)


@pytest.mark.parametrize("block", range(4))
def test_rstream_fuzz(block):
    from dcor import _lib, rstream
    from oracle import oracle as orc
    for cell in _cells(200 + block, 10):
        try:
            ref = orc.rs_sim(cell.to_c(), 3)
        except RuntimeError:
            with pytest.raises(_lib.DcorError):
                rstream.run_grid([cell], 3)
            continue
        got = rstream.run_grid([cell], 3)[0]["records"]
        assert _agree(got, ref), (cell, got, ref)


def test_degenerate_cells_and_empty_launches():
    """n = 1 (no full batch: the oracle's status must be the engine's), zero-replicate
    launches on every kernel family, and cells R itself refuses (n = 0, eps = 0: stopifnot;
    mvrnorm's non-positive-definite Sigma at |rho| > 1; gen_bernoulli's |rho| <= 1;
    alpha >= 2, where mixquant's index ceiling((1-alpha/2)*nsim) < 1) -- refused, never
    launched."""
    from dcor import CellSpec, _lib
    from dcor.sim import simulate
    from oracle import oracle as orc
    for fam, dgp in (("sign", "gaussian"), ("sign", "bernoulli"), ("subG", "bounded_factor"),
                     ("subG", "mix_gaussian")):
        cell = CellSpec(n=1, rho=0.5, eps1=1.0, eps2=1.0, family=fam, dgp=dgp, seed=9)
        try:
            ref = orc.sim_reps(cell.to_c(), 0, 2)
        except RuntimeError:
            with pytest.raises(_lib.DcorError):
                simulate(cell, 2).cpu()
        else:
            assert _agree(simulate(cell, 2).cpu().numpy(), ref), (cell, ref)
        empty = simulate(CellSpec(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family=fam, dgp=dgp, seed=9), 0)
        assert tuple(empty.shape) == (0, 6)
    bad = (dict(n=0), dict(eps1=0.0), dict(eps2=-1.0), dict(alpha=2.0), dict(alpha=float("nan")),
           dict(rho=1.5), dict(dgp="bernoulli", rho=-1.5), dict(family="subG", dgp="mix_gaussian", rho=2.0))
    for kw in bad:
        base = dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", seed=9)
        base.update(kw)
        with pytest.raises(RuntimeError):
            orc.sim_reps(CellSpec(**base).to_c(), 0, 1)
        with pytest.raises(_lib.DcorError):
            simulate(CellSpec(**base), 4).cpu()


@pytest.mark.parametrize("kw", [
    dict(alpha=1.0),                      # qnorm(.5) = 0, log(1/alpha) = 0: zero-width CIs
    dict(alpha=1.0, ci_mode="laplace"),
    dict(alpha=0.0),                      # qnorm(1) = Inf: CIs clipped to [-1, 1] (or NaN at se = 0)
    dict(alpha=1.5),                      # inverted intervals, mixquant element ceiling(.25 nsim)
    dict(alpha=-0.1),                     # qnorm(1.05) = NaN, mixquant index past nsim: NA CIs
    dict(family="subG", dgp="bounded_factor", rho=-0.2),   # sqrt(3 rho) = NaN: runif NaN draws
    dict(family="sign", dgp="bounded_factor", rho=1.3),    # sqrt(3 (1 - rho)) = NaN
    dict(family="subG", alpha=1.0),
])
def test_r_semantics_edge_cells(kw):
    """Cells R evaluates without error although they are degenerate: the engine returns R's
    values (the oracle's), not a refusal (ver-cor-subG.R:57,101,148-152; vert-cor.R:242,302-308)."""
    from dcor import CellSpec
    from dcor.sim import simulate
    from oracle import oracle as orc
    base = dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", seed=9)
    base.update(kw)
    cell = CellSpec(**base)
    ref = orc.sim_reps(cell.to_c(), 3, 7)
    got = simulate(cell, 4, 3).cpu().numpy()
    assert _agree(got, ref), (kw, got, ref)
    if cell.dgp == "bounded_factor":
        assert np.all(np.isnan(got))
