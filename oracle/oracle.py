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
    "orc_cell_check": (C.c_int, [C.c_void_p]),
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


# ------------------------------------------------------------ R's own streams (f4)
class RsState(C.Structure):
    """R's Mersenne-Twister state (.Random.seed[3:627]) and position."""
    _fields_ = [("mt", C.c_uint32 * 624), ("mti", C.c_int32)]


class RsDraws(C.Structure):
    _fields_ = [("X", _D), ("Y", _D), ("lap_sc", C.c_double * 8), ("lap_ni_x", _D),
                ("lap_ni_y", _D), ("flips", _U8), ("lap_local", _D), ("lap_scalar", C.c_double),
                ("mix_z", _D), ("mix_l", _D), ("has_mix", C.c_int), ("k", C.c_int64)]


_PS = C.POINTER(RsState)
for _n, (_r, _a) in {
    "orc_rs_set_seed": (None, [_PS, C.c_int32]),
    "orc_rs_word": (C.c_uint32, [_PS]),
    "orc_rs_word_unif": (C.c_double, [C.c_uint32]),
    "orc_rs_unif": (C.c_double, [_PS]),
    "orc_rs_norm": (C.c_double, [_PS]),
    "orc_rs_norm_words": (C.c_double, [C.c_uint32, C.c_uint32]),
    "orc_rs_exp": (C.c_double, [_PS]),
    "orc_rs_rbinom1": (C.c_double, [_PS, C.c_double]),
    "orc_rs_runif": (C.c_double, [_PS, C.c_double, C.c_double]),
    "orc_rs_laplace_unit_word": (C.c_double, [C.c_uint32]),
    "orc_rs_log": (C.c_double, [C.c_double]),
    "orc_rs_qnorm5": (C.c_double, [C.c_double]),
    "orc_rs_eigen2": (None, [C.c_double] * 3 + [_D, _D]),
    "orc_rs_mvrnorm_factor": (None, [_D, C.c_double, _D]),
    "orc_rs_geometry": (C.c_int, [C.c_void_p, _I64, C.POINTER(C.c_int)]),
    "orc_rs_draw_rep": (C.c_int, [_PS, C.c_void_p, C.POINTER(RsDraws)]),
    "orc_rs_sim": (C.c_int, [C.c_void_p, C.c_int64, _D]),
    "orc_rs_sample_int": (None, [_PS, C.c_int64, C.c_int64, _I32]),
    "orc_rs_hrs_ni_draws": (None, [C.c_int32, C.c_int64, C.c_int64, C.c_int64, _I32, _D, _D]),
    "orc_rs_hrs_int_draws": (None, [C.c_int32, C.c_int64, C.c_int64, _D, _D, _D, _D]),
}.items():
    _f = getattr(lib, _n)
    _f.restype = _r
    _f.argtypes = _a


def rs_state(seed: int) -> RsState:
    """set.seed(seed)."""
    st = RsState()
    lib.orc_rs_set_seed(C.byref(st), int(seed))
    return st


def rs_stream(seed: int, kind: str, count: int, *args) -> np.ndarray:
    """`count` draws of R's runif/rnorm/rexp/rbinom1/word after set.seed(seed)."""
    st = rs_state(seed)
    f = {"unif": lib.orc_rs_unif, "norm": lib.orc_rs_norm, "exp": lib.orc_rs_exp,
         "rbinom1": lib.orc_rs_rbinom1, "runif": lib.orc_rs_runif, "word": lib.orc_rs_word}[kind]
    out = [f(C.byref(st), *args) for _ in range(count)]
    return np.array(out, dtype=np.uint32 if kind == "word" else np.float64)


def rs_eigen2(a, b, c):
    """eigen(matrix(c(a, b, b, c), 2), symmetric = TRUE) -> (values[2], vectors 2x2)."""
    v = np.zeros(2)
    V = np.zeros(4)
    lib.orc_rs_eigen2(a, b, c, v.ctypes.data_as(_D), V.ctypes.data_as(_D))
    return v, V.reshape(2, 2).T


def rs_mvrnorm_factor(sigma, rho):
    s = np.ascontiguousarray(sigma, dtype=np.float64)
    A = np.zeros(4)
    lib.orc_rs_mvrnorm_factor(s.ctypes.data_as(_D), rho, A.ctypes.data_as(_D))
    return A


def rs_draw_reps(cell_struct, reps: int) -> list:
    """The first `reps` replicates' draws of a cell in R's order, after set.seed(cell.seed)."""
    cp = C.cast(C.pointer(cell_struct), C.c_void_p)
    k = C.c_int64()
    mix = C.c_int()
    st_ = lib.orc_rs_geometry(cp, C.byref(k), C.byref(mix))
    if st_:
        raise RuntimeError(f"oracle status {st_}")
    n, nsim = cell_struct.n, cell_struct.nsim
    st = rs_state(cell_struct.seed)
    out = []
    for _ in range(reps):
        a = {"X": np.zeros(n), "Y": np.zeros(n), "lap_ni_x": np.zeros(k.value),
             "lap_ni_y": np.zeros(k.value), "flips": np.zeros(n, dtype=np.uint8),
             "lap_local": np.zeros(n), "mix_z": np.zeros(nsim), "mix_l": np.zeros(nsim)}
        d = RsDraws()
        for key in ("X", "Y", "lap_ni_x", "lap_ni_y", "lap_local", "mix_z", "mix_l"):
            setattr(d, key, a[key].ctypes.data_as(_D))
        d.flips = a["flips"].ctypes.data_as(_U8)
        s = lib.orc_rs_draw_rep(C.byref(st), cp, C.byref(d))
        if s:
            raise RuntimeError(f"oracle status {s}")
        a["lap_sc"] = np.array(d.lap_sc[:])
        a["lap_scalar"] = d.lap_scalar
        a["has_mix"] = d.has_mix
        a["k"] = d.k
        out.append(a)
    return out


def rs_sim(cell_struct, B: int) -> np.ndarray:
    """run_sim_one's B replicates with R's own streams -> [B, 6]."""
    out = np.zeros((B, 6))
    st = lib.orc_rs_sim(C.cast(C.pointer(cell_struct), C.c_void_p), B, out.ctypes.data_as(_D))
    if st:
        raise RuntimeError(f"oracle status {st}")
    return out


def rs_sample_int(seed: int, n: int, k: int) -> np.ndarray:
    """set.seed(seed); sample.int(n, k) - 1."""
    st = rs_state(seed)
    out = np.zeros(k, dtype=np.int32)
    lib.orc_rs_sample_int(C.byref(st), n, k, out.ctypes.data_as(_I32))
    return out


def rs_hrs_ni_draws(seed: int, n: int, k: int, m: int):
    perm = np.zeros(k * m, dtype=np.int32)
    lx, ly = np.zeros(k), np.zeros(k)
    lib.orc_rs_hrs_ni_draws(seed, n, k, m, perm.ctypes.data_as(_I32), lx.ctypes.data_as(_D),
                            ly.ctypes.data_as(_D))
    return perm, lx, ly


def rs_hrs_int_draws(seed: int, n: int, nsim: int = 2000):
    ll, lc = np.zeros(n), np.zeros(1)
    mz, ml = np.zeros(nsim), np.zeros(nsim)
    lib.orc_rs_hrs_int_draws(seed, n, nsim, ll.ctypes.data_as(_D), lc.ctypes.data_as(_D),
                             mz.ctypes.data_as(_D), ml.ctypes.data_as(_D))
    return ll, float(lc[0]), mz, ml
