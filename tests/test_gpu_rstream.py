"""GPU parity of the R-stream mode against its CPU restatement
(oracle/dcor_rstream.c, pinned to values R prints: tests/test_rstream.py).

Bar: the Mersenne-Twister words and every materialised draw bit-exact; estimators and CI
endpoints within 1e-12 relative (the pre-materialised kernels' bar)."""
import os

import numpy as np
import pytest

from helpers import assert_close

pytestmark = pytest.mark.gpu


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


def _spec(dc, **kw):
    base = dict(n=1000, rho=0.5, eps1=1.0, eps2=1.0, family="sign", dgp="gaussian",
                mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_073)
    base.update(kw)
    return dc.CellSpec(**base)


CELLS = {
    "sign-gauss": dict(),
    "sign-gauss-neg": dict(rho=-0.65, eps1=1.5, eps2=0.5, n=1501, seed=1_000_017),
    "sign-gauss-rho0": dict(rho=0.0, eps1=0.5, eps2=1.5, n=777, seed=1_000_001),
    "sign-bern": dict(dgp="bernoulli", mu=(0, 0), sigma=(1, 1), rho=0.3, n=999, seed=1_000_042),
    "sign-nonorm-laplace": dict(normalise=False, ci_mode="laplace", n=640),
    "subG-bounded": dict(family="subG", dgp="bounded_factor", rho=0.3, n=1001, mu=(0, 0), sigma=(1, 1)),
    "subG-bounded-rho0": dict(family="subG", dgp="bounded_factor", rho=0.0, n=512, mu=(0, 0), sigma=(1, 1)),
    "subG-gauss": dict(family="subG", dgp="gaussian", rho=0.8, n=2048, mu=(0, 0), sigma=(1, 1),
                       eps1=0.2, eps2=0.2, seed=1_000_300),
    "subG-mix": dict(family="subG", dgp="mix_gaussian", rho=0.5, n=3001, mu=(0, 0), sigma=(1, 1),
                     seed=1_000_400),
    "sign-mix-pi.3": dict(dgp="mix_gaussian", rho=-0.4, n=2000, pi_mix=0.3, seed=1_000_401),
    "subG-mix-pi1": dict(family="subG", dgp="mix_gaussian", rho=0.2, n=700, pi_mix=1.0, seed=1_000_402),
    "subG-mix-40000": dict(family="subG", dgp="mix_gaussian", rho=0.3, n=40000, seed=1_000_403),
}


@pytest.mark.parametrize("seed", [1, 42, 1_000_073])
def test_mt_words_bitexact(dc, orc, seed):
    got = dc.rstream.words(seed, 5000)
    want = orc.rs_stream(seed, "word", 5000)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name", list(CELLS))
def test_draws_bitexact(dc, orc, name):
    spec = _spec(dc, **CELLS[name])
    reps = 3
    got = dc.rstream.draws(spec, reps)
    ref = orc.rs_draw_reps(spec.to_c(), reps)
    sub = spec.family == "subG"
    for r in range(reps):
        a, g = ref[r], {k: v[r] for k, v in got.items()}
        np.testing.assert_array_equal(g["X"], a["X"], err_msg=f"X rep {r}")
        np.testing.assert_array_equal(g["Y"], a["Y"], err_msg=f"Y rep {r}")
        np.testing.assert_array_equal(g["lap_ni_x"], a["lap_ni_x"])
        np.testing.assert_array_equal(g["lap_ni_y"], a["lap_ni_y"])
        assert g["lap_scalar"] == a["lap_scalar"]
        if sub:
            np.testing.assert_array_equal(g["lap_local"], a["lap_local"])
        else:
            if spec.normalise:
                np.testing.assert_array_equal(g["lap_ni_sc"], a["lap_sc"][:4])
                np.testing.assert_array_equal(g["lap_int_sc"], a["lap_sc"][4:])
            bits = np.unpackbits(g["flips"].view(np.uint8), bitorder="little")[:spec.n]
            np.testing.assert_array_equal(bits, a["flips"])
        if a["has_mix"]:
            np.testing.assert_array_equal(g["mix_z"], a["mix_z"])
            np.testing.assert_array_equal(g["mix_l"], a["mix_l"])


def test_grid_matches_oracle_replicate_by_replicate(dc, orc):
    specs = [_spec(dc, **kw) for kw in CELLS.values()]
    B = 12
    res = dc.rstream.run_grid(specs, B)
    for spec, r in zip(specs, res):
        ref = orc.rs_sim(spec.to_c(), B)
        assert_close(r["records"], ref, what=str(spec))


@pytest.mark.parametrize("max_chunk", [1, 3, 7])
def test_chunked_streams_are_continuous(dc, orc, max_chunk):
    """Short chunks: the Mersenne-Twister state (.Random.seed) carries over exactly, including
    a chunk ending just behind an exp_rand look-ahead (nsim = 3: the untempered-ring path)."""
    specs = [_spec(dc, **CELLS["sign-gauss"]), _spec(dc, **CELLS["subG-bounded"]),
             _spec(dc, family="subG", dgp="bounded_factor", rho=0.4, n=40, nsim=3, mu=(0, 0),
                   sigma=(1, 1), eps1=2.0, eps2=2.0, seed=77)]
    B = 60
    full = dc.rstream.run_grid(specs, B)
    with dc.variants(DCOR_RS_MAX_CHUNK=str(max_chunk)):
        small = dc.rstream.run_grid(specs, B)
    for spec, a, b in zip(specs, full, small):
        np.testing.assert_array_equal(a["records"], b["records"])
    assert_close(small[2]["records"], orc.rs_sim(specs[2].to_c(), B))


def test_run_sim_one_rng_r(dc, orc):
    res = dc.run_sim_one(n=1000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0),
                         B=20, seed=1_000_073, rng="R")
    ref = orc.rs_sim(_spec(dc).to_c(), 20)
    assert_close(np.stack([res["detail"][k] for k in ("ni_hat", "ni_low", "ni_up", "int_hat",
                                                      "int_low", "int_up")], 1), ref)


def test_distributed_rstream_world1_equals_single(dc):
    """The cell-sharded driver (gloo, world 1 here; the 8-GPU run is the driver's) returns the
    single-GPU accumulators bit for bit."""
    import socket

    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from dcor.dist import run_grid_rstream_distributed
        specs = [_spec(dc, **CELLS["sign-gauss"]), _spec(dc, **CELLS["subG-bounded"])]
        got = run_grid_rstream_distributed(specs, 16)
        ref = dc.rstream.run_grid(specs, 16, detail=False)
        for (ni, it), r in zip(got, ref):
            assert bytes(ni) == bytes(r["accum"][0]) and bytes(it) == bytes(r["accum"][1])
    finally:
        dist.destroy_process_group()


def test_headline_cell_full_size(dc, orc):
    """The BASELINE headline cell (n = 1e5) on R's stream: 2 replicates against the CPU
    restatement (the second one starts where the first one's exp_rand walk ended)."""
    spec = dc.headline_cell()
    res = dc.rstream.run_grid([spec], 2)[0]
    assert_close(res["records"], orc.rs_sim(spec.to_c(), 2))


@pytest.mark.parametrize("kw,status", [(dict(n=5, eps1=0.2, eps2=0.2), 2),          # k < 1 (stopifnot)
                                       (dict(dgp="mix_gaussian", n=70000), 1),        # LDS bound
                                       (dict(seed=2 ** 31), 1)])                      # set.seed range
def test_rstream_rejects_like_the_reference(dc, kw, status):
    from dcor import _lib
    spec = _spec(dc, **kw)
    with pytest.raises(_lib.DcorError) as e:
        dc.rstream.run_grid([spec], 2)
    assert e.value.code == status


def test_rstream_extreme_eps_flips_take_no_words(dc, orc):
    """exp(40)/(exp(40)+1) == 1 in double: rbinom(n, 1, 1) returns 1 without drawing."""
    spec = _spec(dc, eps1=40.0, eps2=1.0, n=500)
    res = dc.rstream.run_grid([spec], 3)[0]
    assert_close(res["records"], orc.rs_sim(spec.to_c(), 3))


JUMP_CELLS = ["sign-gauss", "sign-gauss-neg", "sign-bern", "sign-nonorm-laplace", "subG-bounded",
              "subG-gauss"]


def _with_env(env, fn):
    """fn() with the engine switches `env` set (dcor_set_variant), restored afterwards."""
    from dcor import _lib
    with _lib.variants(**env):
        return fn()


def _jump_specs(dc):
    return [_spec(dc, **CELLS[k]) for k in JUMP_CELLS] + [
        _spec(dc, family="subG", dgp="bounded_factor", rho=0.4, n=40, nsim=3, mu=(0, 0),
              sigma=(1, 1), eps1=2.0, eps2=2.0, seed=77)]


@pytest.mark.parametrize("env", [{}, {"DCOR_RS_MAX_CHUNK": "7"}, {"DCOR_RSJ_TIGHT": "1"}],
                         ids=["one-chunk", "chunks-of-7", "budget-overrun-fallback"])
def test_jump_path_equals_sequential_walk(dc, orc, env):
    """The jump path (segment-parallel generation from MT19937 jump-ahead windows, the walk by
    pointer doubling) returns k_rs_stream's records byte for byte -- across chunks (the
    .Random.seed it leaves) and when a chunk overruns its word budget (k_rs_stream re-walks
    it from the unchanged state)."""
    specs = _jump_specs(dc)
    B = 40
    walk = _with_env({"DCOR_RS_JUMP": "0"}, lambda: dc.rstream.run_grid(specs, B))
    jump = _with_env(dict(env, DCOR_RS_JUMP="1"), lambda: dc.rstream.run_grid(specs, B))
    for spec, a, b in zip(specs, walk, jump):
        np.testing.assert_array_equal(a["records"], b["records"], err_msg=str(spec))
        assert bytes(a["accum"][0]) == bytes(b["accum"][0]) and bytes(a["accum"][1]) == bytes(b["accum"][1])
    for spec, b in zip(specs[:2], jump[:2]):
        assert_close(b["records"][:12], orc.rs_sim(spec.to_c(), 12), what=str(spec))


def test_jump_path_long_single_cell_against_oracle(dc, orc):
    """One cell, 300 replicates (~3e6 words: ~100 jump segments): every replicate against the CPU
    restatement, which walks R's stream word by word."""
    spec = _spec(dc)
    B = 300
    got = _with_env({"DCOR_RS_JUMP": "1"}, lambda: dc.rstream.run_grid([spec], B))[0]
    assert_close(got["records"], orc.rs_sim(spec.to_c(), B))
