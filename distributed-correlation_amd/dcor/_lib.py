"""ctypes binding of include/dcor.h (libdcor.so, built in-tree for gfx950).

The shared object is the product: every compute entry runs on the GPU.  If it is
missing this module raises at import time -- there is no Python/CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DCOR_LIB: an alternative in-tree build of the same library (A/B runs of compile-time variants)
LIB_PATH = os.environ.get("DCOR_LIB") or os.path.join(_HERE, "libdcor.so")

DCOR_OK, DCOR_EINVAL, DCOR_EKLT1, DCOR_EHIP, DCOR_ENOMEM, DCOR_ENODEV, DCOR_EFORK = 0, 1, 2, 3, 4, 5, 6
FAMILY_SIGN, FAMILY_SUBG = 0, 1
DGP_GAUSSIAN, DGP_BERNOULLI, DGP_BOUNDED_FACTOR, DGP_MIX_GAUSSIAN = 0, 1, 2, 3
MODE_AUTO, MODE_NORMAL, MODE_LAPLACE = 0, 1, 2
SITE_DGP_A, SITE_DGP_B, SITE_FLIP, SITE_NI_LAP, SITE_SCALAR, SITE_MIX_Z, SITE_MIX_L, SITE_PERM = 1, 2, 3, 4, 5, 6, 7, 8

_MODES = {"auto": MODE_AUTO, "normal": MODE_NORMAL, "laplace": MODE_LAPLACE}


class DcorError(RuntimeError):
    """A non-zero dcor status; `.code` is the DCOR_E* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"dcor error {code}: {msg}")
        self.code = code


class KLessThanOne(DcorError, ValueError):
    """k = floor(n/m) < 1: the reference's stopifnot(k >= 1)."""


class Cell(C.Structure):
    _fields_ = [
        ("family", C.c_int32), ("dgp", C.c_int32), ("n", C.c_int64),
        ("rho", C.c_double), ("eps1", C.c_double), ("eps2", C.c_double), ("alpha", C.c_double),
        ("mu", C.c_double * 2), ("sigma", C.c_double * 2),
        ("eta1", C.c_double), ("eta2", C.c_double),
        ("normalise", C.c_int32), ("ci_mode", C.c_int32), ("nsim", C.c_int64),
        ("seed", C.c_uint64),
        ("mix_mu0", C.c_double * 2), ("mix_sigma0", C.c_double * 2),
        ("mix_mu1", C.c_double * 2), ("mix_sigma1", C.c_double * 2), ("mix_pi", C.c_double),
    ]


class RepOut(C.Structure):
    _fields_ = [(f, C.c_double) for f in ("ni_hat", "ni_lo", "ni_hi", "int_hat", "int_lo", "int_hi")]


class Accum(C.Structure):
    _fields_ = [("n", C.c_int64), ("n_cover", C.c_int64), ("n_cover_na", C.c_int64),
                ("n_na_est", C.c_int64), ("n_na_ci", C.c_int64), ("reserved", C.c_int64 * 3)] + [
        (f, C.c_double * 2) for f in ("est", "est2", "se2", "len", "lo", "hi")]


class Summary(C.Structure):
    _fields_ = [(f, C.c_double) for f in ("mse", "bias", "var", "coverage", "ci_length")]


_P = C.c_void_p


class PrematSign(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("reps", C.c_int64),
        ("eps1", C.c_double), ("eps2", C.c_double), ("alpha", C.c_double),
        ("normalise", C.c_int32), ("ci_mode", C.c_int32), ("nsim", C.c_int64),
        ("X", _P), ("Y", _P), ("xy_stride", C.c_int64),
        ("lap_ni_sc", _P), ("lap_ni_x", _P), ("lap_ni_y", _P), ("lap_int_sc", _P),
        ("flips", _P), ("lap_z", _P), ("mix_z", _P), ("mix_l", _P),
    ]


class PrematSubg(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("reps", C.c_int64),
        ("eps1", C.c_double), ("eps2", C.c_double), ("eta1", C.c_double), ("eta2", C.c_double),
        ("alpha", C.c_double), ("hrs", C.c_int32), ("reserved", C.c_int32),
        ("lam_x", C.c_double), ("lam_y", C.c_double),
        ("lam_s", C.c_double), ("lam_o", C.c_double), ("lam_r", C.c_double), ("delta", C.c_double),
        ("nsim", C.c_int64),
        ("X", _P), ("Y", _P), ("xy_stride", C.c_int64), ("perm", _P),
        ("lap_ni_x", _P), ("lap_ni_y", _P), ("lap_local", _P), ("lap_central", _P),
        ("mix_z", _P), ("mix_l", _P),
    ]


class HrsSegment(C.Structure):
    """dcor_hrs_segment (include/dcor.h): one (eps, keys, replicate range, output row) of a sweep."""
    _fields_ = [("eps", C.c_double), ("seed_ni", C.c_uint64), ("seed_int", C.c_uint64),
                ("rep_begin", C.c_int64), ("reps", C.c_int64), ("out_row", C.c_int64)]


_D = C.POINTER(C.c_double)
_I64 = C.POINTER(C.c_int64)


class RsDraws(C.Structure):
    """dcor_rs_draws: host buffers of the R-stream mode's materialised draws."""
    _fields_ = [("X", _D), ("Y", _D), ("lap_ni_sc", _D), ("lap_int_sc", _D), ("lap_ni_x", _D),
                ("lap_ni_y", _D), ("flips", C.POINTER(C.c_uint32)), ("lap_local", _D),
                ("lap_scalar", _D), ("mix_z", _D), ("mix_l", _D)]

# name -> (restype, argtypes); this list IS the exported ABI (checked against the header
# by tests/test_abi.py).
SIGNATURES = {
    "dcor_version": (C.c_char_p, []),
    "dcor_source_hash": (C.c_char_p, []),
    "dcor_last_error": (C.c_int, [C.c_char_p, C.c_size_t]),
    "dcor_device_count": (C.c_int, []),
    "dcor_shutdown": (C.c_int, []),
    "dcor_set_variant": (C.c_int, [C.c_char_p, C.c_char_p]),
    "dcor_get_variant": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
    "dcor_alloc_count": (C.c_int64, []),
    "dcor_device_bytes": (C.c_int64, []),
    "dcor_sim_chunking": (C.c_int, [C.POINTER(Cell), C.c_int64, _I64, _I64]),
    "dcor_diag_sign_pass": (C.c_int, [C.POINTER(Cell), C.c_int64, C.c_int64, C.c_int, _P]),
    "dcor_diag_sign_ties": (C.c_int, [C.POINTER(Cell), C.c_int64, C.c_int64, _I64]),
    "dcor_lambda_n": (C.c_double, [C.c_double, C.c_double]),
    "dcor_lambda_int_n": (None, [C.c_double, C.c_double, C.c_double, C.c_double, _D]),
    "dcor_lambda_receiver_from_noise": (C.c_double, [C.c_double] * 4),
    "dcor_lambda_from_priv": (C.c_double, [C.c_double] * 5),
    "dcor_qnorm": (C.c_double, [C.c_double]),
    "dcor_sim_launch": (C.c_int, [C.POINTER(Cell), C.c_int64, C.c_int64, _P, _P]),
    "dcor_accumulate_launch": (C.c_int, [_P, C.c_int64, C.c_double, _P, _P]),
    "dcor_accum_merge": (None, [C.POINTER(Accum), C.POINTER(Accum)]),
    "dcor_accum_finalize": (None, [C.POINTER(Accum), C.c_double, C.POINTER(Summary)]),
    "dcor_grid_run": (C.c_int, [C.POINTER(Cell), C.c_int, C.c_int64, C.POINTER(Accum), C.POINTER(RepOut)]),
    "dcor_grid_launch": (C.c_int, [C.POINTER(Cell), C.c_int, _I64, _I64, _P, _P, _P]),
    "dcor_grid_run_multi": (C.c_int, [C.POINTER(Cell), C.c_int, C.c_int64, C.POINTER(C.c_int), C.c_int,
                                      C.POINTER(Accum), C.POINTER(RepOut)]),
    "dcor_rstream_grid_run": (C.c_int, [C.POINTER(Cell), C.c_int, C.c_int64, C.POINTER(Accum),
                                        C.POINTER(RepOut)]),
    "dcor_rstream_draws": (C.c_int, [C.POINTER(Cell), C.c_int64, C.POINTER(RsDraws)]),
    "dcor_rstream_words": (C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_uint32)]),
    "dcor_rstream_mt_jump": (C.c_int, [C.c_int32, C.c_int64, C.POINTER(C.c_uint32)]),
    "dcor_rstream_hrs_draws": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int32), _P, _P, _P, _P,
                                         _P, _P, _P, _P]),
    "dcor_premat_sign_launch": (C.c_int, [C.POINTER(PrematSign), _P, _P]),
    "dcor_premat_subg_launch": (C.c_int, [C.POINTER(PrematSubg), _P, _P]),
    "dcor_panel_dict_probe": (C.c_int, [_P, _P, C.c_int64, C.POINTER(C.c_int)]),
    "dcor_panel_create": (C.c_int, [_P, _P, C.c_int64, _P, C.POINTER(C.c_void_p)]),
    "dcor_panel_coded": (C.c_int, [_P, C.POINTER(C.c_int)]),
    "dcor_panel_destroy": (C.c_int, [_P]),
    "dcor_premat_subg_panel_launch": (C.c_int, [C.POINTER(PrematSubg), _P, _P, _P]),
    "dcor_hrs_fused_launch": (C.c_int, [C.POINTER(PrematSubg), _P, C.c_uint64, C.c_uint64,
                                        C.c_int64, _P, _P]),
    "dcor_hrs_sweep_launch": (C.c_int, [C.POINTER(PrematSubg), _P, C.POINTER(HrsSegment), C.c_int64,
                                        _P, _P]),
    "dcor_batch_geometry": (C.c_int, [C.c_int64, C.c_double, C.c_double, C.c_int, C.c_int, _I64]),
    "dcor_ci_ni_signbatch": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                       C.c_int, _D, _D, _D, _D]),
    "dcor_ci_int_signflip": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                       C.c_int, C.c_int, _D, C.POINTER(C.c_uint8), C.c_double,
                                       _D, _D, C.c_int64, _D]),
    "dcor_correlation_ni_subg": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                           C.c_double, C.c_double, C.c_int, C.c_double,
                                           C.c_double, C.POINTER(C.c_int32), _D, _D, _D]),
    "dcor_ci_int_subg": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                   C.c_double, C.c_double, C.c_int, C.c_double, C.c_double,
                                   C.c_double, C.c_double, _D, C.c_double, _D, _D, C.c_int64, _D]),
    "dcor_mixquant": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, _D]),
    "dcor_priv_standardize": (C.c_int, [_D, C.c_int64, C.c_double, C.c_double, _D, _D]),
    "dcor_draws_launch": (C.c_int, [C.c_int, C.c_uint64, C.c_int, C.c_int64, C.c_int64, C.c_int64,
                                    _P, _P]),
    "dcor_perm_launch": (C.c_int, [C.c_uint64, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                   _P, _P]),
    "dcor_dgp_launch": (C.c_int, [C.POINTER(Cell), C.c_int64, C.c_int64, _P, _P, _P]),
    "dcor_dp_sd": (C.c_int, [_D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, _D, _D]),
    # R-surface helpers (R/dcor*.R): the GPU half of wrappers that draw with R's own RNG
    "dcor_int_subg_sd_uc": (C.c_int, [_D, _D, C.c_int64, C.c_double, C.c_double, C.c_double,
                                      C.c_double, C.c_int, C.c_double, C.c_double, C.c_double,
                                      C.c_double, _D, _D]),
    "dcor_dp_mean": (C.c_int, [_D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, _D]),
    "dcor_standardize_dp": (C.c_int, [_D, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                                      C.c_double, _D]),
    "dcor_gen_bernoulli": (C.c_int, [_D, _D, C.c_int64, C.c_double, _D, _D]),
    "dcor_gen_bounded_factor": (C.c_int, [_D, _D, _D, C.c_int64, _D, _D]),
    "dcor_mvrnorm": (C.c_int, [_D, C.c_int64, _D, _D, C.c_double, _D, _D]),
    "dcor_mix_gaussian": (C.c_int, [_D, C.c_int64, _D, C.c_int64, C.POINTER(C.c_int32), C.c_double,
                                    _D, _D, _D, _D, _D, _D]),
}


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the gfx950 engine first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no CPU fallback")
    # One HIP runtime per process: torch (the device-memory / stream plumbing) ships its own
    # libamdhip64; loading it before libdcor.so makes the engine bind to that same runtime
    # whichever of `import dcor` / `import torch` the caller writes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    buf = C.create_string_buffer(512)
    lib.dcor_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(status: int) -> None:
    if status != DCOR_OK:
        msg = last_error()
        if status == DCOR_EKLT1:
            raise KLessThanOne(status, msg)
        raise DcorError(status, msg)


def mode_code(mode) -> int:
    if isinstance(mode, int):
        return mode
    if isinstance(mode, (list, tuple)):  # R's match.arg default c("auto", ...) -> first
        mode = mode[0]
    if mode not in _MODES:
        raise ValueError(f"mode must be one of {sorted(_MODES)}")
    return _MODES[mode]


def nan_if_none(x) -> float:
    return math.nan if x is None else float(x)


def set_variant(name, value) -> None:
    """An implementation switch (dcor_set_variant): A/B scripts and tests only.  value None
    restores the default; name None restores every default."""
    check(lib.dcor_set_variant(None if name is None else name.encode(),
                               None if value is None else str(value).encode()))


def get_variant(name: str):
    buf = C.create_string_buffer(256)
    r = lib.dcor_get_variant(name.encode(), buf, 256)
    if r < 0:
        raise DcorError(DCOR_EINVAL, last_error())
    return buf.value.decode() if r == 1 else None


class variants:
    """with dcor.variants(DCOR_TILED="0", ...): switches set for the block, restored after."""

    def __init__(self, **kv):
        self.kv = kv
        self.old = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = get_variant(k)
            set_variant(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_variant(k, v)
        return False


def apply_variant_args(items) -> None:
    """bench scripts' --variant NAME=VALUE arguments."""
    for it in items or ():
        k, _, v = it.partition("=")
        set_variant(k, v)
