"""Independent numpy restatement of the reference estimators (second restatement used
to cross-check the C oracle and to generate tests/golden fixtures).

Written separately from oracle/dcor_oracle.c: long-double sums via numpy's np.longdouble
(pairwise order, not R's sequential order -- agreement is to ~1e-15, not bitwise).
Every function cites the R lines it restates.  Parity status: unpinned (no R here).
"""
import math

import numpy as np
from scipy.stats import norm

LD = np.longdouble


def r_sum(x):
    return float(np.sum(np.asarray(x, dtype=LD)))


def r_mean(x):
    x = np.asarray(x, dtype=np.float64)
    n = LD(len(x))
    s = np.sum(x.astype(LD)) / n
    if np.isfinite(float(s)):
        s = s + np.sum(x.astype(LD) - s) / n
    return float(s)


def r_var(x):
    x = np.asarray(x, dtype=np.float64)
    if len(x) < 2:
        return math.nan
    m = LD(r_mean(x))
    d = x.astype(LD) - m
    return float(np.sum(d * d) / LD(len(x) - 1))


def rmax(a, b):
    return math.nan if (math.isnan(a) or math.isnan(b)) else max(a, b)


def rmin(a, b):
    return math.nan if (math.isnan(a) or math.isnan(b)) else min(a, b)


def clip(x, L):
    return np.maximum(np.minimum(np.asarray(x, dtype=np.float64), L), -L)


def lambda_n(n, eta=1.0):  # ver-cor-subG.R:1
    return rmin(2 * eta * math.sqrt(math.log(n)), 2 * math.sqrt(3))


def lambda_int_n(n, eta_s=1.0, eta_r=1.0, eps_s=1.0):  # ver-cor-subG.R:3-7
    return (rmin(2 * eta_s * math.sqrt(math.log(n)), 2 * math.sqrt(3)),
            5 * rmax(eta_r, 1) * rmin(math.log(n), 6) / (rmin(eps_s, 1)))


def mixquant(z, l, c, p):  # ver-cor-subG.R:8-13 with explicit draws
    x = np.asarray(z) + c * np.asarray(l)
    x = np.sort(x[~np.isnan(x)])
    pos = math.ceil(p * len(z))
    return float(x[pos - 1]) if 1 <= pos <= len(x) else math.nan


def qnorm(p):
    return float(norm.ppf(p))


def priv_standardize(v, eps_norm, L, lap):  # vert-cor.R:322-348
    xc = clip(v, L)
    n = len(xc)
    mu = r_mean(xc) + (2 * L / (n * (eps_norm / 2))) * lap[0]
    m2 = r_mean(xc * xc) + (2 * (L * L) / (n * (eps_norm / 2))) * lap[1]
    sd = math.sqrt(rmax(m2 - mu * mu, 1e-12))
    return (xc - mu) / sd


def ci_ni_signbatch(X, Y, eps1, eps2, alpha, normalise, lap_sc, lap_x, lap_y):  # vert-cor.R:204-255
    n = len(X)
    m = math.ceil(8 / (eps1 * eps2))
    k = math.floor(n / m)
    if k < 1:
        return None
    if normalise:
        L = math.sqrt(2 * math.log(n))
        X = priv_standardize(X, eps1, L, lap_sc[0:2])
        Y = priv_standardize(Y, eps2, L, lap_sc[2:4])
    sx = np.sign(np.asarray(X[: k * m])).reshape(k, m)
    sy = np.sign(np.asarray(Y[: k * m])).reshape(k, m)
    T = np.empty(k)
    for j in range(k):
        xt = r_mean(sx[j]) + (2 / (m * eps1)) * lap_x[j]
        yt = r_mean(sy[j]) + (2 / (m * eps2)) * lap_y[j]
        T[j] = m * xt * yt
    eta = (1 / k) * r_sum(T)
    S = math.sqrt(r_var(T)) if k > 1 else math.nan
    crit = qnorm(1 - alpha / 2)
    return [math.sin(math.pi * eta / 2),
            math.sin(math.pi / 2 * rmax(eta - crit * S / math.sqrt(k), -1)),
            math.sin(math.pi / 2 * rmin(eta + crit * S / math.sqrt(k), 1))]


def ci_int_signflip(X, Y, eps1, eps2, alpha, mode, normalise, lap_sc, flips, lap_z, mix_z, mix_l):
    """vert-cor.R:260-317 (+ correlation_INT_signflip 164-195); mode 0/1/2 = auto/normal/laplace."""
    n = len(X)
    if normalise:
        L = math.sqrt(2 * math.log(n))
        X = priv_standardize(X, eps1, L, lap_sc[0:2])
        Y = priv_standardize(Y, eps2, L, lap_sc[2:4])
    sender_is_X = eps1 >= eps2
    eps_s, eps_r = (eps1, eps2) if sender_is_X else (eps2, eps1)
    es = math.exp(eps_s)
    core = (2.0 * np.asarray(flips, dtype=np.float64) - 1) * np.sign(X) * np.sign(Y)
    Z = (2 * (es + 1) / (n * (es - 1) * eps_r)) * lap_z
    eta0 = (es + 1) / (n * (es - 1)) * r_sum(core) + Z
    rho = math.sin(math.pi * eta0 / 2)
    eta = 1 - math.acos(rho) * 2 / math.pi
    q = (es - 1) / (es + 1)
    s2 = 1 - (q * q) * (eta * eta)
    ratio = (es + 1) / (es - 1)
    se = 1 / math.sqrt(n) * math.sqrt(s2) * ratio
    if mode == 0:
        mode = 1 if math.sqrt(n) * eps_r > 0.5 else 2
    if mode == 1:
        w = mixquant(mix_z, mix_l, 2 / (math.sqrt(n * s2) * eps_r), 1 - alpha / 2) * se
    else:
        w = (2 / (n * eps_r)) * ratio * math.log(1 / alpha)
    return [rho, math.sin(math.pi / 2 * rmax(eta - w, -1)), math.sin(math.pi / 2 * rmin(eta + w, 1))]


def ni_subg(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, hrs=False, lam_x=None, lam_y=None,
            perm=None, lap_x=None, lap_y=None):
    """ver-cor-subG.R:25-62; hrs: real-data-sims.R:115-147."""
    n = len(X)
    l1 = lam_x if (hrs and lam_x is not None) else lambda_n(n, eta1)
    l2 = lam_y if (hrs and lam_y is not None) else lambda_n(n, eta2)
    Xc, Yc = clip(X, l1), clip(Y, l2)
    m = math.ceil(8 / (eps1 * eps2))
    m = n if m > n else m
    k = math.floor(n / m)
    if hrs and k < 2:
        k, m = 2, math.floor(n / 2)
    idx = np.asarray(perm) if hrs else np.arange(k * m)
    xm = Xc[idx].reshape(k, m)
    ym = Yc[idx].reshape(k, m)
    xb = (np.sum(xm.astype(LD), axis=1) / LD(m)).astype(np.float64)   # rowMeans
    yb = (np.sum(ym.astype(LD), axis=1) / LD(m)).astype(np.float64)
    xt = xb + (2 * l1 / (m * eps1)) * np.asarray(lap_x)
    yt = yb + (2 * l2 / (m * eps2)) * np.asarray(lap_y)
    rho = (m / k) * r_sum(xt * yt)
    T = m * xt * yt
    se = math.sqrt(r_var(T)) / math.sqrt(k) if k > 1 else math.nan
    crit = qnorm(1 - alpha / 2)
    return [rho, rmax(rho - crit * se, -1), rmin(rho + crit * se, 1)]


def int_subg(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, hrs=False, lam_s=None, lam_o=None,
             lam_r=None, delta=None, lap_local=None, lap_central=0.0, mix_z=None, mix_l=None):
    """ver-cor-subG.R:67-108; hrs: real-data-sims.R:176-252."""
    n = len(X)
    sx = eps1 >= eps2
    eps_s, eps_r = (eps1, eps2) if sx else (eps2, eps1)
    eta_s, eta_r = (eta1, eta2) if sx else (eta2, eta1)
    S, O = (np.asarray(X), np.asarray(Y)) if sx else (np.asarray(Y), np.asarray(X))
    if not hrs:
        ls, lr = lambda_int_n(n, eta_s, eta_r, eps_s)
        U = (clip(S, ls) + (2 * ls / eps_s) * np.asarray(lap_local)) * O
    else:
        delta = 1 / n if delta is None else delta
        if lam_s is None or lam_o is None:
            lam = lambda_int_n(n, eta_s, eta_r, eps_s)
            lam_s = lam[0] if lam_s is None else lam_s
            lam_o = lambda_n(n, eta2 if sx else eta1) if lam_o is None else lam_o
        ls = lam_s
        lr = lam_r if lam_r is not None else (ls + (2 * ls / eps_s) * math.log(1 / delta)) * lam_o
        U = (clip(S, ls) + (2 * ls / eps_s) * np.asarray(lap_local)) * clip(O, lam_o)
    Uc = clip(U, lr)
    rho = r_mean(Uc) + (2 * lr / (n * eps_r)) * lap_central
    sd = math.sqrt(r_var(Uc))
    crit = qnorm(1 - alpha / 2)
    if not hrs:
        s = 2 * lr / (n * eps_r)
        se_norm = math.sqrt(sd * sd + 2 * (s * s))
        width = mixquant(mix_z, mix_l, 2 / (math.sqrt(n) * sd * eps_r), 1 - alpha / 2) * se_norm / math.sqrt(n)
    elif sd == 0:
        width = crit * math.sqrt(2) * (2 * lr / (n * eps_r))
    else:
        width = mixquant(mix_z, mix_l, (2 * lr) / (math.sqrt(n) * sd * eps_r), 1 - alpha / 2) * (sd / math.sqrt(n))
    return [rho, rmax(rho - width, -1), rmin(rho + width, 1)]


def dp_sd(x, lo, hi, eps1, eps2, lap):  # real-data-sims.R:73-84
    xc = np.minimum(np.maximum(np.asarray(x, dtype=np.float64), lo), hi)
    n = len(xc)
    mu = r_mean(xc) + ((hi - lo) / (n * eps1)) * lap[0]
    m2 = r_mean(xc * xc) + ((hi * hi - lo * lo) / (n * eps2)) * lap[1]
    return [mu, math.sqrt(rmax(m2 - mu * mu, 0.0))]
