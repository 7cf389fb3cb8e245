"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical inputs.

Bar: estimators and CI endpoints within 1e-12 relative (ATOL 1e-13 floor for values
that cancel to 0); integer-valued work (batch sign counts, flip sums, Philox draws)
bit-exact.  Oracle parity status: unpinned (oracle/dcor_oracle.h)."""
import ctypes as C

import numpy as np
import pytest

from helpers import assert_close, sign_case, subg_case

pytestmark = pytest.mark.gpu

EPS_PAIRS = [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5), (0.5, 1.5), (0.2, 0.2)]


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


# --------------------------------------------------------------- RNG streams
@pytest.mark.parametrize("kind,site", [(1, 6), (0, 7), (0, 4), (1, 1)])
def test_draws_bitexact(dc, orc, kind, site):
    import torch
    from dcor import _lib
    seed, r0, reps, count = 1_000_073, 5, 3, 4099
    out = torch.empty((reps, count), dtype=torch.float64, device="cuda")
    _lib.check(_lib.lib.dcor_draws_launch(kind, seed, site, r0, reps, count,
                                          C.c_void_p(out.data_ptr()), None))
    got = out.cpu().numpy()
    for r in range(reps):
        ref = (orc.gen_normals if kind == 1 else orc.gen_laplace)(seed, r0 + r, site, count)
        assert np.array_equal(got[r], ref), f"stream mismatch kind={kind} site={site} rep={r0 + r}"


DGP_CELLS = [
    dict(dgp="gaussian", rho=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0)),
    dict(dgp="gaussian", rho=-0.9, mu=(0.0, 0.0), sigma=(1.0, 1.0)),
    dict(dgp="bernoulli", rho=0.3),
    dict(dgp="bounded_factor", rho=0.4),
    dict(dgp="mix_gaussian", rho=0.6),
]


@pytest.mark.parametrize("spec", DGP_CELLS, ids=lambda d: f"{d['dgp']}-{d['rho']}")
def test_dgp_samples_bitexact(dc, orc, spec):
    """Every DGP's samples (dcor_dgp_launch: Dgp<DGP>::one, the full draw contract) against the
    oracle's gen_xy bit for bit.  The Gaussian cells run 3 x 200,003 samples (1.2e6 normal draws
    of the 1024-layer ziggurat): about 5,100 leave its fast path (wedges, retries) and about 64
    reach the base layer's tail."""
    import torch
    from dcor import _lib
    from dcor.sim import CellSpec
    n = 200_003 if spec["dgp"] == "gaussian" else 20_011
    reps, r0 = 3, 7
    cell = CellSpec(n=n, eps1=1.0, eps2=1.0, family="sign", seed=1_000_011, **spec)
    cs = cell.to_c()
    X = torch.empty((reps, n), dtype=torch.float64, device="cuda")
    Y = torch.empty_like(X)
    _lib.check(_lib.lib.dcor_dgp_launch(C.byref(cs), r0, reps, C.c_void_p(X.data_ptr()),
                                        C.c_void_p(Y.data_ptr()), None))
    gx, gy = X.cpu().numpy(), Y.cpu().numpy()
    for r in range(reps):
        ox, oy = orc.gen_xy(cs, r0 + r)
        assert np.array_equal(gx[r], ox) and np.array_equal(gy[r], oy), f"{spec} rep {r0 + r}"


# ------------------------------------------------------- explicit-input sign
@pytest.mark.parametrize("n", [10, 1000, 10_000, 100_000])
@pytest.mark.parametrize("eps", EPS_PAIRS)
def test_sign_single(dc, orc, n, eps):
    eps1, eps2 = eps
    g = np.random.default_rng(n * 7 + int(eps1 * 10) * 3 + int(eps2 * 10))
    cs = sign_case(g, n, eps1, eps2)
    if cs["k"] >= 1:
        st, ref = orc.ci_ni_signbatch(cs["X"], cs["Y"], eps1, eps2, 0.05, 1, cs["lap_ni_sc"],
                                      cs["lap_x"], cs["lap_y"])
        assert st == 0
        got = dc.ci_NI_signbatch(cs["X"], cs["Y"], eps1, eps2, noise={
            "lap_sc": cs["lap_ni_sc"], "lap_x": cs["lap_x"], "lap_y": cs["lap_y"]})
        assert_close([got["rho_hat"], *got["ci"]], ref, what=f"NI sign n={n} eps={eps}")
    else:
        with pytest.raises(dc.KLessThanOne):
            dc.ci_NI_signbatch(cs["X"], cs["Y"], eps1, eps2, noise={
                "lap_sc": cs["lap_ni_sc"], "lap_x": cs["lap_x"], "lap_y": cs["lap_y"]})
    for mode in (0, 1, 2):
        st, ref, md = orc.ci_int_signflip(cs["X"], cs["Y"], eps1, eps2, 0.05, mode, 1,
                                          cs["lap_int_sc"], cs["flips"], cs["lap_z"],
                                          cs["mix_z"], cs["mix_l"])
        assert st == 0
        got = dc.ci_INT_signflip(cs["X"], cs["Y"], eps1, eps2, mode=["auto", "normal", "laplace"][mode],
                                 noise={"lap_sc": cs["lap_int_sc"], "flips": cs["flips"],
                                        "lap_z": cs["lap_z"], "mix_z": cs["mix_z"],
                                        "mix_l": cs["mix_l"]})
        assert_close([got["rho_hat"], *got["ci"]], ref, what=f"INT sign n={n} eps={eps} mode={mode}")
        assert got["mode"] == ("normal" if md == 1 else "laplace")


# ------------------------------------------------------- explicit-input sub-G
@pytest.mark.parametrize("n", [10, 1000, 10_000, 100_000])
@pytest.mark.parametrize("eps", EPS_PAIRS)
@pytest.mark.parametrize("hrs", [False, True])
def test_subg_single(dc, orc, n, eps, hrs):
    eps1, eps2 = eps
    g = np.random.default_rng(n * 11 + int(eps1 * 10) * 5 + int(eps2 * 10) + 999 * hrs)
    cs = subg_case(g, n, eps1, eps2, nsim=2000 if hrs else 1000, hrs=hrs)
    lamx, lamy = (2.2, 2.6) if hrs else (np.nan, np.nan)
    st, ref, km = orc.ni_subg(cs["X"], cs["Y"], eps1, eps2, hrs=int(hrs), lam_x=lamx, lam_y=lamy,
                              perm=cs["perm"], lap_x=cs["lap_x"], lap_y=cs["lap_y"])
    assert st == 0
    got = dc.correlation_NI_subG(cs["X"], cs["Y"], eps1, eps2, hrs=hrs,
                                 lambda_X=None if not hrs else lamx,
                                 lambda_Y=None if not hrs else lamy, perm=cs["perm"],
                                 noise={"lap_x": cs["lap_x"], "lap_y": cs["lap_y"]})
    assert_close([got["rho_hat"], *got["ci"]], ref, what=f"NI subG n={n} eps={eps} hrs={hrs}")
    kw = dict(lam_s=2.2, lam_o=2.6) if hrs else {}
    st, ref, lam = orc.int_subg(cs["X"], cs["Y"], eps1, eps2, hrs=int(hrs), lap_local=cs["lap_local"],
                                lap_central=cs["lap_central"], mix_z=cs["mix_z"], mix_l=cs["mix_l"], **kw)
    assert st == 0
    got = dc.ci_INT_subG(cs["X"], cs["Y"], eps1, eps2, hrs=hrs,
                         lambda_sender=kw.get("lam_s"), lambda_other=kw.get("lam_o"),
                         noise={"lap_local": cs["lap_local"], "lap_central": cs["lap_central"],
                                "mix_z": cs["mix_z"], "mix_l": cs["mix_l"]})
    assert_close([got["rho_hat"], *got["ci"]], ref, what=f"INT subG n={n} eps={eps} hrs={hrs}")


# ------------------------------------------------------------ fused engine
FUSED_CELLS = [
    dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)),
    dict(n=4000, rho=0.9, eps1=1.5, eps2=0.5, family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)),
    dict(n=3000, rho=0.0, eps1=0.5, eps2=1.5, family="sign", dgp="gaussian"),
    dict(n=2000, rho=0.3, eps1=1.0, eps2=1.0, family="sign", dgp="bernoulli"),
    dict(n=2500, rho=0.65, eps1=1.5, eps2=0.5, family="subG", dgp="bounded_factor"),
    dict(n=2500, rho=0.3, eps1=0.5, eps2=0.5, family="subG", dgp="gaussian"),
    dict(n=1600, rho=0.8, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", ci_mode="laplace"),
    dict(n=1000, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", normalise=False),
    # gen_mix_gaussian (ver-cor-subG.R:113-133): R defaults, and a non-dyadic pi_mix
    dict(n=5500, rho=0.6, eps1=5.0, eps2=1.0, family="subG", dgp="mix_gaussian"),
    dict(n=3001, rho=0.4, eps1=1.0, eps2=1.0, family="sign", dgp="mix_gaussian", pi_mix=0.3,
         mix_mu1=(0.5, -0.5), mix_sigma1=(0.7, 1.3)),
    dict(n=2000, rho=0.2, eps1=1.0, eps2=1.0, family="sign", dgp="mix_gaussian", normalise=False),
]


@pytest.mark.parametrize("spec", FUSED_CELLS)
def test_fused_vs_oracle(dc, orc, spec):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(seed=1_000_000 + spec["n"] % 97, **spec)
    got = simulate(cell, 24, rep_begin=3).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 3, 27)
    assert_close(got, ref, what=f"fused {spec}")


# Bernoulli sign cells run the bit-plane kernel: batch sizes m = 1, 2, 8, 11, 32, 128,
# n off the 256-sample chunk grid, normalise = FALSE, the Laplace CI mode.
BERN_CELLS = [
    dict(n=1000, rho=0.5, eps1=4.0, eps2=4.0),     # m = 1
    dict(n=777, rho=0.9, eps1=2.0, eps2=2.0),      # m = 2
    dict(n=2049, rho=0.0, eps1=1.0, eps2=1.0),     # m = 8, tail
    dict(n=3001, rho=0.65, eps1=1.5, eps2=0.5),    # m = 11
    dict(n=1500, rho=0.3, eps1=0.5, eps2=0.5),     # m = 32
    dict(n=1300, rho=0.8, eps1=0.25, eps2=0.25),   # m = 128, k < 256
    dict(n=999, rho=0.4, eps1=1.0, eps2=1.0, normalise=False),
    dict(n=1200, rho=0.15, eps1=1.0, eps2=1.0, ci_mode="laplace"),
]


@pytest.mark.parametrize("spec", BERN_CELLS)
def test_bernoulli_planes_vs_oracle(dc, orc, spec):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(seed=2_000_003 + spec["n"], family="sign", dgp="bernoulli", **spec)
    got = simulate(cell, 20, rep_begin=5).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 5, 25)
    assert_close(got, ref, what=f"bernoulli planes {spec}")


@pytest.mark.parametrize("eps", [(1.0, 1.0), (1.5, 0.5), (0.5, 0.5)])
def test_bernoulli_planes_vs_regen(dc, eps, variant):
    """Bit-plane kernel == per-sample regenerate kernel, bit for bit (clip(1) = 1 makes
    the DP-mean sums integers in both)."""
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=30_011, rho=0.5, eps1=eps[0], eps2=eps[1], family="sign", dgp="bernoulli",
                    seed=77)
    a = simulate(cell, 64).cpu().numpy()
    variant("DCOR_SIGN_KERNEL", "regen")
    b = simulate(cell, 64).cpu().numpy()
    assert np.array_equal(a, b, equal_nan=True)


def test_fused_split_invariance(dc):
    """Per-replicate results do not depend on how the replicate range is split."""
    from dcor.sim import headline_cell, simulate
    cell = headline_cell(20_000)
    a = simulate(cell, 96).cpu().numpy()
    b = np.concatenate([simulate(cell, 40, 0).cpu().numpy(), simulate(cell, 56, 40).cpu().numpy()])
    assert np.array_equal(a, b)


# C3 size (n = 1e6, the grids' largest n): every fused kernel family
# against the oracle fed the same Philox streams, replicates 7 and 8 of each cell.
C3_CELLS = [
    dict(rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)),
    dict(rho=0.8, eps1=1.5, eps2=0.5, family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)),
    dict(rho=0.15, eps1=0.5, eps2=0.5, family="sign", dgp="gaussian", mu=(0.5, 0.5), sigma=(2.0, 2.0)),  # m = 32
    dict(rho=0.3, eps1=1.0, eps2=1.0, family="sign", dgp="bernoulli"),
    dict(rho=0.65, eps1=0.5, eps2=1.5, family="subG", dgp="bounded_factor"),
    dict(rho=0.6, eps1=1.0, eps2=1.0, family="subG", dgp="mix_gaussian"),
]


@pytest.mark.parametrize("spec", C3_CELLS)
def test_fused_vs_oracle_n1e6(dc, orc, spec):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=1_000_000, seed=1_000_211, **spec)
    got = simulate(cell, 2, rep_begin=7).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 7, 9)
    assert_close(got, ref, what=f"fused n=1e6 {spec}")


def test_fused_split_invariance_n1e6(dc):
    """At n = 1e6 a replicate's result is the same alone or inside a larger launch."""
    from dcor.sim import headline_cell, simulate
    cell = headline_cell(1_000_000)
    a = simulate(cell, 12).cpu().numpy()
    b = np.concatenate([simulate(cell, 5, 0).cpu().numpy(), simulate(cell, 7, 5).cpu().numpy()])
    assert np.array_equal(a, b)
    assert np.all(np.isfinite(a))
    assert np.all((a[:, 1] <= a[:, 2]) & (a[:, 4] <= a[:, 5]))


# Clip-saturated and degenerate Gaussian cells: the record-code window sits on E[clip(x)], the
# private centres beside it, so samples pinned at the clip bound L tie a centre's code far more
# often (each tie is regenerated exactly).  mu far outside [-L, L] clips every sample to +-L; a
# near-zero sigma puts every sample at mu; sigma_x != sigma_y and rho = -1 stress the window per
# coordinate.  Both kernel forms: the wave kernel (n <= 16384) and the workgroup kernel.
SATURATED_CELLS = [
    dict(n=20_000, rho=0.5, eps1=1.0, eps2=1.0, mu=(10.0, -10.0), sigma=(1.0, 1.0)),
    dict(n=4_000, rho=0.5, eps1=1.0, eps2=1.0, mu=(10.0, 0.5), sigma=(1.0, 2.0)),
    dict(n=30_000, rho=0.0, eps1=1.0, eps2=1.0, mu=(0.25, 0.25), sigma=(1e-9, 1e-9)),
    dict(n=25_000, rho=-1.0, eps1=1.5, eps2=0.5, mu=(0.0, 3.0), sigma=(3.0, 0.5)),
    # batch sizes off the m = 8 loop (the unit stream): m = 32 in the wave kernel, m = 11 in the
    # workgroup kernel, both with clip-saturated coordinates
    dict(n=6_000, rho=0.3, eps1=0.5, eps2=0.5, mu=(10.0, 0.5), sigma=(1.0, 2.0)),
    dict(n=50_000, rho=0.5, eps1=1.5, eps2=0.5, mu=(-10.0, 10.0), sigma=(1.0, 1.0)),
]


@pytest.mark.parametrize("spec", SATURATED_CELLS)
def test_saturated_cells_vs_oracle(dc, orc, spec):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(seed=3_000_011 + spec["n"], **spec)
    got = simulate(cell, 6, rep_begin=2).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 2, 8)
    assert_close(got, ref, what=f"saturated {spec}")


# The workgroup Gaussian pass 1 compacts its slow samples into a per-wave list every four loop
# steps and regenerates them in-kernel: n % 4 != 0 puts slow samples in the tail group, and n
# just above a multiple of the 512-group loop step leaves waves with different step counts
# (partial quads).
@pytest.mark.parametrize("n", [16_387, 100_003, 2_048 * 4 * 4 + 4 * 64 + 2, 131_071])
def test_fused_vs_oracle_bitmap_geometry(dc, orc, n):
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=n, rho=0.4, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=5_000_000 + n)
    got = simulate(cell, 4, rep_begin=3).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 3, 7)
    assert_close(got, ref, what=f"bitmap geometry n={n}")


# Batch sizes above 252 take pass 2's record-by-record exact path (dcor_fused.hip, m > 252), in the
# wave kernels (n <= 16384) and in the workgroup kernels: eps 0.1 x 0.1 gives m = 800,
# eps 0.16 x 0.16 m = 313; through dcor_sim_launch and through the batched grid.
M_BIG_CELLS = [dict(n=12_000, eps1=0.1, eps2=0.1), dict(n=20_000, eps1=0.1, eps2=0.1),
               dict(n=9_391, eps1=0.16, eps2=0.16), dict(n=40_001, eps1=0.16, eps2=0.16, dgp="bernoulli")]


@pytest.mark.parametrize("spec", M_BIG_CELLS)
def test_fused_vs_oracle_m_over_252(dc, orc, spec):
    from dcor.sim import CellSpec, run_grid, simulate
    cell = CellSpec(rho=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=6_000_000 + spec["n"],
                    **{"dgp": "gaussian", **spec})
    k, m = dc.api.batch_geometry(cell.n, cell.eps1, cell.eps2, "sign")
    assert m > 252 and k >= 10
    got = simulate(cell, 8, rep_begin=5).cpu().numpy()
    ref = orc.sim_reps(cell.to_c(), 5, 13)
    assert_close(got, ref, what=f"m={m} {spec}")
    grid = run_grid([cell], 13, detail=True, devices=[0])[0]["records"]
    np.testing.assert_array_equal(grid[5:13].view(np.int64), got.view(np.int64))
