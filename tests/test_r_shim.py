"""The R binding without R: every .Call in R/dcor*.R names a routine registered in src/dcor_r.c
with the same argument count; the shim compiles (against the stub R API in tests/rstub/, built by
__graft_entry__.build() with -Wall -Werror) and its routines run through the stub runtime --
host-side routines here, GPU routines in tests/test_gpu_rsurface.py -- with R's argument
passing and R's error path (Rf_error after dcor_last_error)."""
import math
import os
import re

import numpy as np
import pytest

from rstub_py import RError, RStub

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RDIR = os.path.join(ROOT, "distributed-correlation_amd", "R")
RSRC = "".join(open(os.path.join(RDIR, f), encoding="utf-8").read()
               for f in ("dcor.R", "dcor_subG.R", "dcor_hrs.R"))
CSRC = open(os.path.join(ROOT, "distributed-correlation_amd", "src", "dcor_r.c")).read()
HDR = open(os.path.join(ROOT, "include", "dcor.h")).read()


def _call_args(src):
    """{routine: argument count} for every .Call("name", ...) (balanced parentheses)."""
    out = {}
    for m in re.finditer(r'\.Call\("(\w+)"', src):
        i, depth, args = m.end(), 1, 0  # counts the commas after the routine name
        while depth:
            ch = src[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == "," and depth == 1:
                args += 1
            i += 1
        assert out.get(m.group(1), args) == args, m.group(1)
        out[m.group(1)] = args
    return out


def test_call_sites_match_registration():
    reg = {n: int(k) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', CSRC)}
    calls = _call_args(RSRC)
    assert calls, "no .Call sites found"
    for name, nargs in calls.items():
        assert name in reg, f"{name} called from R but not registered"
        assert reg[name] == nargs, f"{name}: R passes {nargs}, registered {reg[name]}"
    assert set(reg) == set(calls), set(reg) ^ set(calls)


def test_registered_signatures_have_that_many_sexps():
    reg = {n: int(k) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', CSRC)}
    for name, k in reg.items():
        m = re.search(r"SEXP " + name + r"\(([^)]*)\)", CSRC)
        assert m, name
        assert m.group(1).count("SEXP") == k, name


def test_shim_calls_only_declared_entry_points():
    body = re.sub(r"/\*.*?\*/", "", CSRC, flags=re.S)
    used = set(re.findall(r"\b(dcor_(?!R_)\w+)\s*\(", body))
    used -= set(re.findall(r"\b(?:static\s+)?\w+\s+(dcor_\w+)\s*\([^;]*\)\s*\{", body))  # shim helpers
    declared = set(re.findall(r"\b(dcor_\w+)\s*\(", re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)))
    assert used <= declared, used - declared
    assert {"dcor_rstream_grid_run", "dcor_grid_run_multi"} <= used


@pytest.fixture(scope="module")
def rs():
    return RStub()


def test_stub_registration_matches_source(rs):
    reg = {n: int(k) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', CSRC)}
    for name, k in reg.items():
        assert rs.nargs(name) == k


def test_host_routines_through_the_shim(rs):
    """Closed forms evaluated on the host: lambda_n, lambda_INT_n (ver-cor-subG.R:1-7),
    lambda_from_priv, lambda_receiver_from_noise (real-data-sims.R:103-106,170-174)."""
    assert rs.value(rs.call("dcor_R_lambda_n", rs.real(1e5), rs.real(1.0)))[0] == 2 * math.sqrt(3)
    lam = rs.value(rs.call("dcor_R_lambda_INT_n", rs.real(1e5), rs.real(1.0), rs.real(1.0), rs.real(0.5)))
    assert lam[0] == 2 * math.sqrt(3) and lam[1] == 5 * 1 * 6 / 0.5
    got = rs.value(rs.call("dcor_R_lambda_from_priv", rs.real(45), rs.real(90), rs.real(65.0),
                           rs.real(10.0), rs.real(1e-8)))[0]
    assert got == 2.5
    got = rs.value(rs.call("dcor_R_lambda_receiver_from_noise", rs.real(2.0), rs.real(3.0),
                           rs.real(2.0), rs.real(1e-4)))[0]
    assert got == (2.0 + (2 * 2.0 / 2.0) * math.log(1 / 1e-4)) * 3.0


def test_error_path_is_rf_error(rs):
    """A failing entry surfaces through Rf_error with dcor_last_error's message (R's stop()),
    after the shim released everything it allocated (R_alloc'd scratch is freed by the jump)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("host without a GPU only: the entry must fail with DCOR_ENODEV")
    z = rs.real(np.zeros(5))
    with pytest.raises(RError, match="status 5"):
        rs.call("dcor_R_mixquant", z, z, rs.real(1.0), rs.real(0.975))
    with pytest.raises(ValueError):
        rs.call("dcor_R_mixquant", z, z)          # wrong arity: not callable
