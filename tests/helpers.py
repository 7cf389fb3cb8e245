"""Shared test helpers: tolerance, seeded explicit-input cases."""
import math

import numpy as np

RTOL = 1e-12   # north_star: estimators and CI endpoints within 1e-12 relative (fp64)
ATOL = 1e-13   # absolute floor for values that cancel towards 0 (SURVEY §7.3 hard part 1)


def close(a, b, rtol=RTOL, atol=ATOL):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    diff = np.abs(a - b)
    ok = (diff <= atol + rtol * np.maximum(np.abs(a), np.abs(b))) | both_nan | (a == b)
    return bool(np.all(ok))


def assert_close(a, b, rtol=RTOL, atol=ATOL, what=""):
    if not close(a, b, rtol, atol):
        a = np.asarray(a, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        raise AssertionError(f"{what}: mismatch\n got {a!r}\n ref {b!r}\n diff {np.abs(a-b)!r}")


def unit_laplace(g, size):
    u = g.uniform(-0.5, 0.5, size)
    return -np.sign(u) * np.log1p(-2.0 * np.abs(u))


def geometry(n, eps1, eps2, subg=False, hrs=False):
    m = math.ceil(8.0 / (eps1 * eps2))
    if subg and m > n:
        m = n
    k = math.floor(n / m)
    if hrs and k < 2:
        k, m = 2, math.floor(n / 2)
    return k, m


def sign_case(g, n, eps1, eps2, rho=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), nsim=1000):
    """Explicit inputs of one sign-family replicate (NI + INT)."""
    cov = [[sigma[0] ** 2, sigma[0] * sigma[1] * rho], [sigma[0] * sigma[1] * rho, sigma[1] ** 2]]
    xy = g.multivariate_normal(mu, cov, size=n)
    k, m = geometry(n, eps1, eps2)
    eps_s = max(eps1, eps2)
    p = math.exp(eps_s) / (math.exp(eps_s) + 1)
    return dict(X=xy[:, 0].copy(), Y=xy[:, 1].copy(), lap_ni_sc=unit_laplace(g, 4),
                lap_x=unit_laplace(g, max(k, 0)), lap_y=unit_laplace(g, max(k, 0)),
                lap_int_sc=unit_laplace(g, 4), flips=g.binomial(1, p, n).astype(np.uint8),
                lap_z=float(unit_laplace(g, 1)[0]), mix_z=g.standard_normal(nsim),
                mix_l=unit_laplace(g, nsim), k=k, m=m)


def subg_case(g, n, eps1, eps2, rho=0.5, nsim=1000, hrs=False):
    cU, cE = math.sqrt(3 * rho), math.sqrt(3 * (1 - rho))
    U = g.uniform(-cU, cU, n)
    X = U + g.uniform(-cE, cE, n)
    Y = U + g.uniform(-cE, cE, n)
    k, m = geometry(n, eps1, eps2, subg=True, hrs=hrs)
    perm = g.permutation(n)[: k * m].astype(np.int32) if hrs else None
    return dict(X=X, Y=Y, lap_x=unit_laplace(g, k), lap_y=unit_laplace(g, k),
                lap_local=unit_laplace(g, n), lap_central=float(unit_laplace(g, 1)[0]),
                mix_z=g.standard_normal(nsim), mix_l=unit_laplace(g, nsim), perm=perm, k=k, m=m)
