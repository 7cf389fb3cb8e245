"""CPU consistency checks of the R binding (R is not installed here, so the shim cannot be
compiled or run): every .Call in R/dcor.R names a routine registered in src/dcor_r.c with the
same argument count, each registered routine's C signature has that many SEXP parameters,
and every dcor_* function the shim calls is declared in include/dcor.h."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RSRC = open(os.path.join(ROOT, "distributed-correlation_amd", "R", "dcor.R")).read()
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
        out[m.group(1)] = args
    return out


def test_call_sites_match_registration():
    reg = {n: int(k) for n, k in re.findall(r'\{"(\w+)", \(DL_FUNC\)&\w+, (\d+)\}', CSRC)}
    calls = _call_args(RSRC)
    assert calls, "no .Call sites found"
    for name, nargs in calls.items():
        assert name in reg, f"{name} called from R but not registered"
        assert reg[name] == nargs, f"{name}: R passes {nargs}, registered {reg[name]}"


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
    assert "dcor_rstream_grid_run" in used
