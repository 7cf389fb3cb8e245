"""ctypes wrapper of the CPU oracle (oracle/build/libdcor_oracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product.  Parity status: unpinned (see
dcor_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libdcor_oracle.so")

if not os.path.exists(_SO):
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)

lib = C.CDLL(_SO)
_D = C.POINTER(C.c_double)
_I32 = C.POINTER(C.c_int32)
_U8 = C.POINTER(C.c_uint8)
_U32 = C.POINTER(C.c_uint32)
_I64 = C.POINTER(C.c_int64)

_sigs = {
    "orc_r_sum": (C.c_double, [_D, C.c_int64]),
    "orc_r_mean": (C.c_double, [_D, C.c_int64]),
    "orc_r_var": (C.c_double, [_D, C.c_int64]),
    "orc_qnorm": (C.c_double, [C.c_double]),
    "orc_lambda_n": (C.c_double, [C.c_double, C.c_double]),
    "orc_lambda_int_n": (None, [C.c_double] * 4 + [_D]),
    "orc_mixquant": (C.c_double, [_D, _D, C.c_int64, C.c_double, C.c_double]),
    "orc_priv_standardize": (None, [_D, C.c_int64, C.c_double, C.c_double, _D, _D]),
    "orc_ci_ni_signbatch": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                      C.c_int, _D, _D, _D, _D]),
    "orc_ci_int_signflip": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                      C.c_int, C.c_int, _D, _U8, C.c_double, _D, _D, C.c_int64,
                                      _D, C.POINTER(C.c_int)]),
    "orc_ni_subg": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                              C.c_double, C.c_int, C.c_double, C.c_double, _I32, _D, _D, _D, _I64]),
    "orc_int_subg": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                               C.c_double, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                               _D, C.c_double, _D, _D, C.c_int64, _D, _D]),
    "orc_dp_mean": (C.c_double, [_D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double]),
    "orc_dp_sd": (None, [_D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, _D, _D]),
    "orc_lambda_from_priv": (C.c_double, [C.c_double] * 4),
    "orc_lambda_receiver_from_noise": (C.c_double, [C.c_double] * 4),
    "orc_mvrnorm_factor": (None, [_D, _D, C.c_double, _D]),
    "orc_gen_xy": (None, [C.c_void_p, C.c_int64, _D, _D]),
    "orc_mvrnorm_apply": (None, [_D, _D, C.c_int64, _D, _D, _D, _D]),
    "orc_gen_bernoulli": (None, [_D, _D, C.c_int64, C.c_double, _D, _D]),
    "orc_gen_bounded_factor": (None, [_D, _D, _D, C.c_int64, C.c_double, _D, _D]),
    "orc_philox4x32_10": (None, [_U32, C.c_uint32, C.c_uint32, _U32]),
    "orc_u53": (C.c_double, [C.c_uint32, C.c_uint32]),
    "orc_log": (C.c_double, [C.c_double]),
    "orc_sincospi": (None, [C.c_double, _D, _D]),
    "orc_unit_laplace": (C.c_double, [C.c_double]),
    "orc_sim_rep": (C.c_int, [C.c_void_p, C.c_int64, _D]),
    "orc_sim_reps": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int, _D]),
    "orc_gen_normals": (None, [C.c_uint64, C.c_int64, C.c_int, C.c_int64, _D]),
    "orc_gen_laplace": (None, [C.c_uint64, C.c_int64, C.c_int, C.c_int64, _D]),
    "orc_perm": (None, [C.c_uint64, C.c_int, C.c_int64, C.c_int64, C.c_int64, _I32]),
}
for _n, (_r, _a) in _sigs.items():
    _f = getattr(lib, _n)
    _f.restype = _r
    _f.argtypes = _a


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_D)


def r_sum(x):
    a, p = _d(x)
    return lib.orc_r_sum(p, len(a))


def r_mean(x):
    a, p = _d(x)
    return lib.orc_r_mean(p, len(a))


def r_var(x):
    a, p = _d(x)
    return lib.orc_r_var(p, len(a))


def qnorm(p):
    return lib.orc_qnorm(float(p))


def lambda_n(n, eta=1.0):
    return lib.orc_lambda_n(float(n), float(eta))


def lambda_int_n(n, eta_s=1.0, eta_r=1.0, eps_s=1.0):
    out = np.zeros(2)
    lib.orc_lambda_int_n(float(n), float(eta_s), float(eta_r), float(eps_s), out.ctypes.data_as(_D))
    return out


def mixquant(z, l, c, p):
    z, pz = _d(z)
    l, pl = _d(l)
    return lib.orc_mixquant(pz, pl, len(z), float(c), float(p))


def priv_standardize(v, eps, L, lap):
    v, pv = _d(v)
    lap, pl = _d(lap)
    out = np.empty_like(v)
    lib.orc_priv_standardize(pv, len(v), float(eps), float(L), pl, out.ctypes.data_as(_D))
    return out


def ci_ni_signbatch(X, Y, eps1, eps2, alpha, normalise, lap_sc, lap_x, lap_y):
    X, px = _d(X)
    Y, py = _d(Y)
    sc, ps = _d(lap_sc)
    lx, plx = _d(lap_x)
    ly, ply = _d(lap_y)
    out = np.zeros(3)
    st = lib.orc_ci_ni_signbatch(px, py, len(X), eps1, eps2, alpha, int(normalise), ps, plx, ply,
                                 out.ctypes.data_as(_D))
    return st, out


def ci_int_signflip(X, Y, eps1, eps2, alpha, mode, normalise, lap_sc, flips, lap_z, mix_z, mix_l):
    X, px = _d(X)
    Y, py = _d(Y)
    sc, ps = _d(lap_sc)
    fl = np.ascontiguousarray(flips, dtype=np.uint8)
    mz, pmz = _d(mix_z)
    ml, pml = _d(mix_l)
    out = np.zeros(3)
    md = C.c_int(0)
    st = lib.orc_ci_int_signflip(px, py, len(X), eps1, eps2, alpha, int(mode), int(normalise), ps,
                                 fl.ctypes.data_as(_U8), float(lap_z), pmz, pml, len(mz),
                                 out.ctypes.data_as(_D), C.byref(md))
    return st, out, md.value


def ni_subg(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, hrs=0, lam_x=np.nan, lam_y=np.nan,
            perm=None, lap_x=None, lap_y=None):
    X, px = _d(X)
    Y, py = _d(Y)
    lx, plx = _d(lap_x)
    ly, ply = _d(lap_y)
    pm = None
    if perm is not None:
        perm = np.ascontiguousarray(perm, dtype=np.int32)
        pm = perm.ctypes.data_as(_I32)
    out = np.zeros(3)
    km = np.zeros(2, dtype=np.int64)
    st = lib.orc_ni_subg(px, py, len(X), eps1, eps2, eta1, eta2, alpha, int(hrs), lam_x, lam_y,
                         pm, plx, ply, out.ctypes.data_as(_D), km.ctypes.data_as(_I64))
    return st, out, km


def int_subg(X, Y, eps1, eps2, eta1=1.0, eta2=1.0, alpha=0.05, hrs=0, lam_s=np.nan,
             lam_o=np.nan, lam_r=np.nan, delta=np.nan, lap_local=None, lap_central=0.0,
             mix_z=None, mix_l=None):
    X, px = _d(X)
    Y, py = _d(Y)
    ll, pll = _d(lap_local)
    mz, pmz = _d(mix_z)
    ml, pml = _d(mix_l)
    out = np.zeros(3)
    lam = np.zeros(3)
    st = lib.orc_int_subg(px, py, len(X), eps1, eps2, eta1, eta2, alpha, int(hrs), lam_s, lam_o,
                          lam_r, delta, pll, float(lap_central), pmz, pml, len(mz),
                          out.ctypes.data_as(_D), lam.ctypes.data_as(_D))
    return st, out, lam


def dp_sd(x, lo, hi, eps1, eps2, lap):
    x, pxx = _d(x)
    lap, pl = _d(lap)
    out = np.zeros(2)
    lib.orc_dp_sd(pxx, len(x), lo, hi, eps1, eps2, pl, out.ctypes.data_as(_D))
    return out


def philox(ctr, k0, k1):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib.orc_philox4x32_10(c.ctypes.data_as(_U32), k0, k1, o.ctypes.data_as(_U32))
    return o


def gen_normals(seed, rep, site, count):
    z = np.zeros(count)
    lib.orc_gen_normals(seed, rep, site, count, z.ctypes.data_as(_D))
    return z


def gen_laplace(seed, rep, site, count):
    z = np.zeros(count)
    lib.orc_gen_laplace(seed, rep, site, count, z.ctypes.data_as(_D))
    return z


def sim_reps(cell_struct, r0, r1, threads=1):
    """Fused replicates [r0, r1) of a dcor_cell (ctypes struct) -> [r1-r0, 6]."""
    out = np.zeros((r1 - r0, 6))
    st = lib.orc_sim_reps(C.cast(C.pointer(cell_struct), C.c_void_p), r0, r1, threads,
                          out.ctypes.data_as(_D))
    if st:
        raise RuntimeError(f"oracle status {st}")
    return out


def perm(seed, site, rep, n, count):
    out = np.zeros(count, dtype=np.int32)
    lib.orc_perm(seed, site, rep, n, count, out.ctypes.data_as(_I32))
    return out


def gen_xy(cell_struct, rep):
    """DGP draws (X, Y) of replicate `rep` of a dcor_cell (ctypes struct)."""
    X = np.zeros(cell_struct.n)
    Y = np.zeros(cell_struct.n)
    lib.orc_gen_xy(C.cast(C.pointer(cell_struct), C.c_void_p), rep, X.ctypes.data_as(_D),
                   Y.ctypes.data_as(_D))
    return X, Y
