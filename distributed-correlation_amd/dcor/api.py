"""R-surface mirror of the reference's estimator functions (host side of the C-ABI).

Same names, argument meaning, defaults, return shapes and error behaviour as the R
closures they replace; each call runs on the GPU through libdcor.so.  Where the R
function draws its own noise from the global R RNG, these take an optional
`noise=` dict of unit-scale draws (the explicit-input contract of include/dcor.h)
and otherwise draw it from a numpy Generator (`rng=`, default: the module RNG that
`set_seed` resets, the analogue of R's set.seed).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

from . import _lib
from ._lib import C, check, lib

_rng = np.random.default_rng(2025)


def set_seed(seed: int) -> None:
    """Analogue of R's set.seed for the host-side noise draws."""
    global _rng
    _rng = np.random.default_rng(seed)


def _g(rng):
    return _rng if rng is None else rng


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


# ----------------------------------------------------------------- unit draws
def unit_laplace(size, rng=None) -> np.ndarray:
    """extraDistr::rlaplace(size, 0, 1): -sign(u)*log(1-2|u|), u ~ U(-1/2, 1/2)."""
    u = _g(rng).uniform(-0.5, 0.5, size)
    return -np.sign(u) * np.log1p(-2.0 * np.abs(u))


def rLap(n: int = 1, scale: float = 1.0, rng=None) -> np.ndarray:
    """rLap (vert-cor.R:106 / real-data-sims.R:58-61)."""
    return scale * unit_laplace(n, rng)


def mix_draws(nsim: int, rng=None):
    """rnorm(nsim), rexp(nsim)*(2*rbinom(nsim,1,.5)-1) (ver-cor-subG.R:11)."""
    g = _g(rng)
    z = g.standard_normal(nsim)
    l = g.exponential(1.0, nsim) * (2.0 * g.binomial(1, 0.5, nsim) - 1.0)
    return z, l


# -------------------------------------------------------------- calibration
def lambda_n(n, eta=1.0) -> float:
    """lambda_n (ver-cor-subG.R:1)."""
    return lib.dcor_lambda_n(float(n), float(eta))


def lambda_INT_n(n, eta_s=1.0, eta_r=1.0, eps_s=1.0) -> np.ndarray:
    """lambda_INT_n (ver-cor-subG.R:3-7) -> c(lambda_s, lambda_r)."""
    out = np.zeros(2)
    lib.dcor_lambda_int_n(float(n), float(eta_s), float(eta_r), float(eps_s), _dp(out))
    return out


def lambda_receiver_from_noise(lambda_sender, lambda_other, eps_sender, delta_per_sample) -> float:
    """real-data-sims.R:170-174."""
    return lib.dcor_lambda_receiver_from_noise(float(lambda_sender), float(lambda_other),
                                               float(eps_sender), float(delta_per_sample))


def lambda_from_priv(lo, hi, priv, eps_sd=1e-8) -> float:
    """real-data-sims.R:103-106 (priv = {'mean', 'sd'})."""
    return lib.dcor_lambda_from_priv(float(lo), float(hi), float(priv["mean"]), float(priv["sd"]),
                                     float(eps_sd))


def qnorm(p) -> float:
    return lib.dcor_qnorm(float(p))


def batch_geometry(n, eps1, eps2, family="sign", hrs=False):
    """(k, m) as the estimators compute them."""
    km = np.zeros(2, dtype=np.int64)
    fam = _lib.FAMILY_SUBG if family == "subG" else _lib.FAMILY_SIGN
    st = lib.dcor_batch_geometry(int(n), float(eps1), float(eps2), fam, int(bool(hrs)),
                                 km.ctypes.data_as(C.POINTER(C.c_int64)))
    check(st)
    return int(km[0]), int(km[1])


# ---------------------------------------------------------------- mixquant
def mixquant(c, p, nsim: int = 1000, z=None, l=None, rng=None) -> float:
    """mixquant (ver-cor-subG.R:8-13; nsim=2000 in real-data-sims.R:161-164)."""
    if z is None or l is None:
        z, l = mix_draws(nsim, rng)
    z, l = _f64(z), _f64(l)
    out = C.c_double()
    check(lib.dcor_mixquant(_dp(z), _dp(l), len(z), float(c), float(p), C.byref(out)))
    return out.value


# ------------------------------------------------------- DP helper functions
def priv_standardize(vec, eps_norm, L_raw=6.0, lap=None, rng=None) -> np.ndarray:
    """priv_standardize (vert-cor.R:322-348): the DP mean / second-moment helper."""
    v = _f64(vec)
    lap = _f64(unit_laplace(2, rng) if lap is None else lap)
    out = np.empty_like(v)
    check(lib.dcor_priv_standardize(_dp(v), len(v), float(eps_norm), float(L_raw), _dp(lap), _dp(out)))
    return out


def dp_sd(x, lo, hi, eps1, eps2, lap=None, rng=None) -> dict:
    """dp_sd (real-data-sims.R:73-84) -> {'mean', 'sd'} (NA dropped like x[!is.na(x)])."""
    v = _f64(x)
    v = np.ascontiguousarray(v[~np.isnan(v)])
    if v.size == 0:
        return {"mean": math.nan, "sd": math.nan}
    lap = _f64(unit_laplace(2, rng) if lap is None else lap)
    out = np.zeros(2)
    check(lib.dcor_dp_sd(_dp(v), len(v), float(lo), float(hi), float(eps1), float(eps2), _dp(lap), _dp(out)))
    return {"mean": float(out[0]), "sd": float(out[1])}


def dp_mean(x, lo, hi, eps, lap=None, rng=None) -> float:
    """dp_mean (real-data-sims.R:64-70) (NA dropped like x[!is.na(x)])."""
    v = _f64(x)
    v = np.ascontiguousarray(v[~np.isnan(v)])
    if v.size == 0:
        return math.nan
    lap1 = unit_laplace(1, rng)[0] if lap is None else float(np.ravel(lap)[0])
    out = C.c_double()
    check(lib.dcor_dp_mean(_dp(v), len(v), float(lo), float(hi), float(eps), float(lap1), C.byref(out)))
    return out.value


def standardize_dp(x, priv, lo, hi, eps=1e-8) -> np.ndarray:
    """standardize_dp (real-data-sims.R:87-90): (pmin(pmax(x, lo), hi) - mean) / max(sd, eps)."""
    v = _f64(x)
    out = np.empty_like(v)
    check(lib.dcor_standardize_dp(_dp(v), len(v), float(lo), float(hi), float(priv["mean"]),
                                  float(priv["sd"]), float(eps), _dp(out)))
    return out


# ----------------------------------------------- DGPs from explicit (R) draws
# The arithmetic half of the R wrappers' generators (R/dcor*.R): the caller supplies the draws R
# would make, in R's order; the GPU returns (X, Y) as R computes them.
def gen_bernoulli(u, v, rho):
    """gen_bernoulli (vert-cor.R:78-98) from u = runif(n), v = runif(n) -> (X, Y)."""
    u, v = _f64(u), _f64(v)
    X, Y = np.empty_like(u), np.empty_like(u)
    check(lib.dcor_gen_bernoulli(_dp(u), _dp(v), len(u), float(rho), _dp(X), _dp(Y)))
    return X, Y


def gen_bounded_factor(U, E1, E2):
    """gen_bounded_factor (ver-cor-subG.R:141-154): (U + E1, U + E2) from its runif draws."""
    U, E1, E2 = _f64(U), _f64(E1), _f64(E2)
    X, Y = np.empty_like(U), np.empty_like(U)
    check(lib.dcor_gen_bounded_factor(_dp(U), _dp(E1), _dp(E2), len(U), _dp(X), _dp(Y)))
    return X, Y


def mvrnorm(z, mu, sigma, rho):
    """MASS::mvrnorm(n, mu, Sigma(sigma, rho)) (vert-cor.R:389-394) from z = rnorm(2n)."""
    z = _f64(z)
    n = len(z) // 2
    mu_, sg = _f64(mu), _f64(sigma)
    X, Y = np.empty(n), np.empty(n)
    check(lib.dcor_mvrnorm(_dp(z), n, _dp(mu_), _dp(sg), float(rho), _dp(X), _dp(Y)))
    return X, Y


def mix_gaussian(z0, z1, perm, rho, mu0=(0, 0), sigma0=(1, 1), mu1=(3, 3), sigma1=(2, 0.5)):
    """gen_mix_gaussian (ver-cor-subG.R:115-136) from z0 = rnorm(2 n0), z1 = rnorm(2 n1) and the
    0-based row order perm = sample.int(n) - 1."""
    z0, z1 = _f64(z0), _f64(z1)
    n0, n1 = len(z0) // 2, len(z1) // 2
    pm = np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
    a = [_f64(v) for v in (mu0, sigma0, mu1, sigma1)]
    X, Y = np.empty(n0 + n1), np.empty(n0 + n1)
    check(lib.dcor_mix_gaussian(_dp(z0), n0, _dp(z1), n1, pm.ctypes.data_as(C.POINTER(C.c_int32)),
                                float(rho), *[_dp(v) for v in a], _dp(X), _dp(Y)))
    return X, Y


# ---------------------------------------------------------------- sign family
def ci_NI_signbatch(X, Y, eps1, eps2, alpha=0.05, normalise=True, noise: Optional[dict] = None,
                    rng=None) -> dict:
    """ci_NI_signbatch (vert-cor.R:204-255) -> {'rho_hat', 'ci'}.

    noise: {'lap_sc': [mu_X, m2_X, mu_Y, m2_Y], 'lap_x': [k], 'lap_y': [k]} unit Laplace."""
    X, Y = _f64(X), _f64(Y)
    if len(X) != len(Y):
        raise _lib.DcorError(_lib.DCOR_EINVAL, "length(X) == length(Y) is not TRUE")
    n = len(X)
    m = math.ceil(8.0 / (eps1 * eps2))
    k = int(math.floor(n / m)) if m > 0 else 0
    if noise is None:
        g = _g(rng)
        noise = {"lap_sc": unit_laplace(4, g), "lap_x": unit_laplace(max(k, 0), g),
                 "lap_y": unit_laplace(max(k, 0), g)}
    sc, lx, ly = _f64(noise["lap_sc"]), _f64(noise["lap_x"]), _f64(noise["lap_y"])
    out = np.zeros(3)
    check(lib.dcor_ci_ni_signbatch(_dp(X), _dp(Y), n, float(eps1), float(eps2), float(alpha),
                                   int(bool(normalise)), _dp(sc), _dp(lx), _dp(ly), _dp(out)))
    return {"rho_hat": float(out[0]), "ci": out[1:3].copy()}


def ci_INT_signflip(X, Y, eps1, eps2, alpha=0.05, mode=("auto", "normal", "laplace"),
                    normalise=True, noise: Optional[dict] = None, nsim: int = 1000, rng=None) -> dict:
    """ci_INT_signflip (vert-cor.R:260-317) -> {'rho_hat', 'ci', 'mode', 'roles'}.

    noise: {'lap_sc': [4], 'flips': [n] in {0,1}, 'lap_z': float, 'mix_z': [nsim], 'mix_l': [nsim]}."""
    X, Y = _f64(X), _f64(Y)
    if len(X) != len(Y) or not (eps1 > 0 and eps2 > 0):
        raise _lib.DcorError(_lib.DCOR_EINVAL, "stopifnot(length(X) == length(Y), eps1 > 0, eps2 > 0)")
    n = len(X)
    md = _lib.mode_code(mode)
    sender_is_X = eps1 >= eps2
    eps_s, eps_r = (eps1, eps2) if sender_is_X else (eps2, eps1)
    if noise is None:
        g = _g(rng)
        p = math.exp(eps_s) / (math.exp(eps_s) + 1)
        z, l = mix_draws(nsim, g)
        noise = {"lap_sc": unit_laplace(4, g), "flips": g.binomial(1, p, n),
                 "lap_z": float(unit_laplace(1, g)[0]), "mix_z": z, "mix_l": l}
    sc = _f64(noise["lap_sc"])
    fl = np.ascontiguousarray(np.asarray(noise["flips"], dtype=np.uint8))
    mz, ml = _f64(noise["mix_z"]), _f64(noise["mix_l"])
    out = np.zeros(3)
    check(lib.dcor_ci_int_signflip(_dp(X), _dp(Y), n, float(eps1), float(eps2), float(alpha), md,
                                   int(bool(normalise)), _dp(sc),
                                   fl.ctypes.data_as(C.POINTER(C.c_uint8)), float(noise["lap_z"]),
                                   _dp(mz), _dp(ml), len(mz), _dp(out)))
    resolved = md if md != _lib.MODE_AUTO else (
        _lib.MODE_NORMAL if math.sqrt(n) * eps_r > 0.5 else _lib.MODE_LAPLACE)
    return {"rho_hat": float(out[0]), "ci": out[1:3].copy(),
            "mode": "normal" if resolved == _lib.MODE_NORMAL else "laplace",
            "roles": "X→Y" if sender_is_X else "Y→X"}


def correlation_INT_signflip(X, Y, eps1, eps2, noise=None, rng=None) -> float:
    """correlation_INT_signflip (vert-cor.R:164-195) on already-normalised X, Y."""
    return ci_INT_signflip(X, Y, eps1, eps2, mode="laplace", normalise=False,
                           noise=noise, rng=rng)["rho_hat"]


# ---------------------------------------------------------------- sub-G family
def correlation_NI_subG(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, lambda_X=None,
                        lambda_Y=None, hrs: bool = False, perm=None, noise: Optional[dict] = None,
                        rng=None) -> dict:
    """correlation_NI_subG: ver-cor-subG.R:25-62, or (hrs=True) real-data-sims.R:115-147
    with lambda overrides, the k<2 guard and random batches idx = sample.int(n, k*m).

    noise: {'lap_x': [k], 'lap_y': [k]}; perm (hrs): 0-based sample.int(n, k*m) - 1."""
    X, Y = _f64(X), _f64(Y)
    if hrs:
        ok = ~(np.isnan(X) | np.isnan(Y))
        X, Y = np.ascontiguousarray(X[ok]), np.ascontiguousarray(Y[ok])
    if len(X) != len(Y):
        raise _lib.DcorError(_lib.DCOR_EINVAL, "n == length(Y) is not TRUE")
    n = len(X)
    k, m = batch_geometry(n, eps1, eps2, "subG", hrs)
    g = _g(rng)
    if hrs and perm is None:
        perm = g.permutation(n)[: k * m]
    if noise is None:
        noise = {"lap_x": unit_laplace(k, g), "lap_y": unit_laplace(k, g)}
    lx, ly = _f64(noise["lap_x"]), _f64(noise["lap_y"])
    pm = None if perm is None else np.ascontiguousarray(np.asarray(perm, dtype=np.int32))
    out = np.zeros(3)
    check(lib.dcor_correlation_ni_subg(
        _dp(X), _dp(Y), n, float(eps1), float(eps2), float(eta1), float(eta2), float(alpha),
        int(bool(hrs)), _lib.nan_if_none(lambda_X), _lib.nan_if_none(lambda_Y),
        None if pm is None else pm.ctypes.data_as(C.POINTER(C.c_int32)), _dp(lx), _dp(ly), _dp(out)))
    res = {"rho_hat": float(out[0]), "ci": out[1:3].copy()}
    if hrs:
        res.update(k=k, m=m,
                   lambda_X=lambda_X if lambda_X is not None else lambda_n(n, eta1),
                   lambda_Y=lambda_Y if lambda_Y is not None else lambda_n(n, eta2))
    return res


def ci_INT_subG(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, mode=("auto", "normal", "laplace"),
                lambda_sender=None, lambda_other=None, lambda_receiver=None, delta_clip=None,
                hrs: bool = False, noise: Optional[dict] = None, nsim: Optional[int] = None,
                rng=None) -> dict:
    """ci_INT_subG: ver-cor-subG.R:67-108, or (hrs=True) real-data-sims.R:176-252.

    noise: {'lap_local': [n], 'lap_central': float, 'mix_z': [nsim], 'mix_l': [nsim]}."""
    X, Y = _f64(X), _f64(Y)
    if hrs:
        ok = ~(np.isnan(X) | np.isnan(Y))
        X, Y = np.ascontiguousarray(X[ok]), np.ascontiguousarray(Y[ok])
    if len(X) != len(Y):
        raise _lib.DcorError(_lib.DCOR_EINVAL, "n == length(Y) is not TRUE")
    n = len(X)
    if nsim is None:
        nsim = 2000 if hrs else 1000
    if noise is None:
        g = _g(rng)
        z, l = mix_draws(nsim, g)
        noise = {"lap_local": unit_laplace(n, g), "lap_central": float(unit_laplace(1, g)[0]),
                 "mix_z": z, "mix_l": l}
    ll, mz, ml = _f64(noise["lap_local"]), _f64(noise["mix_z"]), _f64(noise["mix_l"])
    out = np.zeros(3)
    check(lib.dcor_ci_int_subg(
        _dp(X), _dp(Y), n, float(eps1), float(eps2), float(eta1), float(eta2), float(alpha),
        int(bool(hrs)), _lib.nan_if_none(lambda_sender), _lib.nan_if_none(lambda_other),
        _lib.nan_if_none(lambda_receiver), _lib.nan_if_none(delta_clip), _dp(ll),
        float(noise["lap_central"]), _dp(mz), _dp(ml), len(mz), _dp(out)))
    sender_is_X = eps1 >= eps2
    res = {"rho_hat": float(out[0]), "ci": out[1:3].copy(), "roles": "X→Y" if sender_is_X else "Y→X"}
    if not hrs:
        res["mode"] = mode
    else:
        eps_s = eps1 if sender_is_X else eps2
        delta = 1.0 / n if delta_clip is None else delta_clip
        ls, lo_ = lambda_sender, lambda_other
        if ls is None or lo_ is None:
            lam = lambda_INT_n(n, eta1 if sender_is_X else eta2, eta2 if sender_is_X else eta1, eps_s)
            ls = lam[0] if ls is None else ls
            lo_ = lambda_n(n, eta2 if sender_is_X else eta1) if lo_ is None else lo_
        lr = lambda_receiver if lambda_receiver is not None else lambda_receiver_from_noise(ls, lo_, eps_s, delta)
        res.update(lambda_sender=ls, lambda_other=lo_, lambda_receiver=lr, delta_clip=delta)
    return res
