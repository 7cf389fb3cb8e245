"""CPU tests of the drop-in boundary: libdcor.so loads, exports every function
include/dcor.h declares, struct layouts match the ctypes mirror, host-side calibration
scalars follow the R formulas, and compute entries fail loudly without a GPU."""
import ctypes as C
import math
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dcor.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dcor_\w+)\s*\(", txt)))


def test_header_functions_exported_and_bound():
    from dcor import _lib
    names = declared_functions()
    assert len(names) >= 24
    so = C.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(so, n), f"{n} declared in dcor.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} not bound in dcor/_lib.py"
    assert set(_lib.SIGNATURES) == set(names)


def test_exports_are_c_symbols():
    from dcor import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (dcor_\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_struct_layout_matches_header():
    """Compile a tiny C program against include/dcor.h and compare sizeof/offsetof."""
    from dcor import _lib
    structs = {"dcor_cell": _lib.Cell, "dcor_rep_out": _lib.RepOut, "dcor_accum": _lib.Accum,
               "dcor_summary": _lib.Summary, "dcor_premat_sign": _lib.PrematSign,
               "dcor_premat_subg": _lib.PrematSubg, "dcor_rs_draws": _lib.RsDraws,
               "dcor_hrs_segment": _lib.HrsSegment}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    got = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, f"{cname}.{fname}"


def test_host_calibration_matches_r_formulas():
    import dcor
    for n in (10, 20, 21, 404, 1e4, 1e5, 1e6):
        assert dcor.lambda_n(n) == min(2 * math.sqrt(math.log(n)), 2 * math.sqrt(3))
        for eps_s in (0.5, 1.0, 1.5):
            ls, lr = dcor.lambda_INT_n(n, 1, 1, eps_s)
            assert ls == min(2 * math.sqrt(math.log(n)), 2 * math.sqrt(3))
            assert lr == 5 * 1 * min(math.log(n), 6) / min(eps_s, 1)
    from oracle.oracle import lib as olib
    assert dcor.qnorm(0.975) == olib.orc_rs_qnorm5(0.975)  # R's qnorm: AS241, same operation order
    assert abs(dcor.qnorm(0.975) - 1.959963984540054) <= 4.5e-16
    # real-data-sims.R:170-174, 103-106
    assert dcor.lambda_receiver_from_noise(2.0, 3.0, 2.0, 1e-4) == (2.0 + (2 * 2.0 / 2.0) * math.log(1e4)) * 3.0
    assert dcor.lambda_from_priv(45, 90, {"mean": 65.0, "sd": 10.0}) == 2.5


def test_batch_geometry():
    import dcor
    from dcor.api import batch_geometry
    assert batch_geometry(100_000, 1.0, 1.0) == (12500, 8)
    assert batch_geometry(100_000, 1.5, 0.5) == (9090, 11)
    assert batch_geometry(100_000, 0.5, 0.5) == (3125, 32)
    assert batch_geometry(5, 0.2, 0.2, "subG") == (1, 5)          # m > n -> m = n
    assert batch_geometry(9, 0.5, 0.5, "subG", hrs=True) == (2, 4)  # k < 2 guard
    with pytest.raises(dcor.KLessThanOne):
        batch_geometry(5, 0.2, 0.2, "sign")


@pytest.mark.skipif(os.environ.get("DCOR_ASSUME_GPU") == "1", reason="GPU present")
def test_compute_fails_loudly_without_gpu():
    import dcor
    from dcor import _lib
    if _lib.lib.dcor_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(dcor.DcorError) as e:
        dcor.mixquant(1.0, 0.975)
    assert e.value.code == _lib.DCOR_ENODEV
    with pytest.raises(dcor.DcorError):
        dcor.ci_NI_signbatch(np.ones(100), np.ones(100), 1.0, 1.0)
    c = dcor.CellSpec(n=100, rho=0.5, eps1=1, eps2=1).to_c()
    assert _lib.lib.dcor_sim_launch(C.byref(c), 0, 1, C.c_void_p(8), None) == _lib.DCOR_ENODEV


def test_argument_validation_without_gpu():
    """Validation happens before any device access (the reference's stopifnot)."""
    import dcor
    with pytest.raises(dcor.DcorError):
        dcor.ci_INT_signflip(np.ones(3), np.ones(4), 1.0, 1.0)
    with pytest.raises(dcor.DcorError):
        dcor.ci_INT_signflip(np.ones(3), np.ones(3), 0.0, 1.0)


def test_hrs_sweep_argument_checks_without_gpu():
    """dcor_hrs_sweep_launch rejects null arguments before any device access."""
    from dcor import _lib
    base = _lib.PrematSubg(n=10, hrs=1, delta=0.1, nsim=10)
    seg = (_lib.HrsSegment * 1)(_lib.HrsSegment(eps=1.0, reps=1))
    assert _lib.lib.dcor_hrs_sweep_launch(None, None, seg, 1, C.c_void_p(8), None) == _lib.DCOR_EINVAL
    assert _lib.lib.dcor_hrs_sweep_launch(C.byref(base), None, seg, 1, C.c_void_p(8), None) == _lib.DCOR_EINVAL


def test_accum_merge_and_finalize_host():
    """dcor_accum_merge / finalize are host helpers: mse, bias, var, coverage, ci_length."""
    from dcor import _lib
    from dcor.sim import finalize, merge
    g = np.random.default_rng(5)
    est = g.normal(0.5, 0.1, 1000)
    lo, hi = est - 0.2, est + 0.2
    accs = []
    for part in np.array_split(np.arange(1000), 3):
        a = _lib.Accum()
        a.n = len(part)
        cov = (0.5 >= lo[part]) & (0.5 <= hi[part])
        a.n_cover = int(cov.sum())
        for name, vals in (("est", est[part]), ("est2", est[part] ** 2), ("se2", (est[part] - 0.5) ** 2),
                           ("len", hi[part] - lo[part]), ("lo", lo[part]), ("hi", hi[part])):
            getattr(a, name)[0] = math.fsum(vals)
        accs.append(a)
    s = finalize(merge(accs), 0.5)
    assert abs(s["mse"] - np.mean((est - 0.5) ** 2)) < 1e-15
    assert abs(s["bias"] - (np.mean(est) - 0.5)) < 1e-15
    assert abs(s["var"] - np.var(est, ddof=1)) < 1e-13
    assert s["coverage"] == np.mean((0.5 >= lo) & (0.5 <= hi))
    assert abs(s["ci_length"] - 0.4) < 1e-15


def test_sim_chunking_plan_without_gpu():
    """dcor_sim_chunking is planning only (no device): the one-pass sign path splits the headline's
    8192 replicates into four chunks of 2048 (the shape bench.py times its live ceilings at), always
    at least two chunks from 512 replicates, equal chunks covering every replicate; other kernel
    families take one launch."""
    from dcor import _lib
    from dcor.sim import CellSpec, headline_cell

    def plan(cell, reps):
        ch, nc = C.c_int64(), C.c_int64()
        _lib.check(_lib.lib.dcor_sim_chunking(C.byref(cell.to_c()), reps, C.byref(ch), C.byref(nc)))
        return ch.value, nc.value

    assert plan(headline_cell(), 8192) == (2048, 4)
    assert plan(headline_cell(), 512) == (256, 2)
    for n, reps in ((100_000, 10_001), (1_000_000, 100_000), (20_000, 3)):
        ch, nc = plan(headline_cell(n), reps)
        assert nc >= 1 and ch * nc >= reps and ch * (nc - 1) < reps
    bern = CellSpec(n=100_000, rho=0.5, eps1=1.0, eps2=1.0, dgp="bernoulli", mu=(0.0, 0.0), sigma=(1.0, 1.0))
    assert plan(bern, 8192) == (8192, 1)
    assert plan(headline_cell(), 0) == (0, 0)
