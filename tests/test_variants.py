"""The engine's implementation switches (dcor_set_variant, include/dcor.h): the library reads no
environment variable, so a replicate's bits are a function of (cell, seed, replicate) alone -- the
per-cell set.seed reproducibility contract of vert-cor.R:364.  CPU: the sources never call getenv,
and the switch table's ABI.  GPU (test_gpu_variants.py): every former variable set to a non-default
value leaves the headline, C5 and C5-continuous results unchanged."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed-correlation_amd", "csrc")

# every switch the engine knows (dcor_capi.cpp kVariantNames)
SWITCHES = {
    "DCOR_SIGN_KERNEL": "regen", "DCOR_CODE_WINDOW": "wide", "DCOR_SIGN_PIPELINE": "0",
    "DCOR_SIGN_XCALL": "0", "DCOR_SIGN_P2E": "0", "DCOR_EPILOGUE": "block", "DCOR_HRS_FUSED_L2": "1",
    "DCOR_HRS_WPE": "4", "DCOR_PREMAT_PIPELINE": "1", "DCOR_DICT_VARIANT": "2", "DCOR_L2_VARIANT": "3",
    "DCOR_TILED": "0", "DCOR_TILED_VARIANT": "0", "DCOR_TILED_INT": "2", "DCOR_GRID_CHUNK_ITEMS": "4096",
    "DCOR_GRID_SLAB_MB": "1", "DCOR_GRID_MIN_CHUNKS": "9", "DCOR_GRID_REC_MB": "1", "DCOR_RS_JUMP": "0",
    "DCOR_RS_BUDGET_MB": "64", "DCOR_RS_MAX_CHUNK": "3", "DCOR_RSJ_TIGHT": "1",
}


def test_engine_sources_read_no_environment():
    hits = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".cpp", ".hip", ".h")):
            for i, line in enumerate(open(os.path.join(CSRC, f)), 1):
                if re.search(r"\b(getenv|secure_getenv|environ)\b", line):
                    hits.append(f"{f}:{i}: {line.strip()}")
    assert not hits, "engine reads the environment:\n" + "\n".join(hits)


def test_switch_table_matches_sources():
    src = open(os.path.join(CSRC, "dcor_capi.cpp")).read()
    table = src[src.index("kVariantNames[] = {"):src.index("};", src.index("kVariantNames[] = {"))]
    names = set(re.findall(r'"(DCOR_[A-Z0-9_]+)"', table))
    assert names == set(SWITCHES)
    used = set()
    for f in os.listdir(CSRC):
        if f.endswith((".cpp", ".hip")):
            used |= set(re.findall(r'(?:variant|env_size)\("(DCOR_[A-Z0-9_]+)"', open(os.path.join(CSRC, f)).read()))
    assert used == names, f"read but not in the table: {used - names}; in the table, never read: {names - used}"


def test_set_and_get_variant():
    from dcor import _lib
    assert all(_lib.get_variant(k) is None for k in SWITCHES)
    with _lib.variants(DCOR_TILED="0", DCOR_CODE_WINDOW="4,8"):
        assert _lib.get_variant("DCOR_TILED") == "0"
        assert _lib.get_variant("DCOR_CODE_WINDOW") == "4,8"
    assert _lib.get_variant("DCOR_TILED") is None and _lib.get_variant("DCOR_CODE_WINDOW") is None
    _lib.set_variant("DCOR_RS_JUMP", "1")
    _lib.set_variant(None, None)
    assert _lib.get_variant("DCOR_RS_JUMP") is None
    with pytest.raises(_lib.DcorError):
        _lib.set_variant("DCOR_NO_SUCH_SWITCH", "1")
    with pytest.raises(_lib.DcorError):
        _lib.get_variant("HOME")


def test_environment_does_not_set_switches():
    """A variable in the caller's environment is not a switch."""
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = %r; from dcor import _lib; "
            "print(all(_lib.get_variant(k) is None for k in %r))") % (
        [ROOT, os.path.join(ROOT, "distributed-correlation_amd")], sorted(SWITCHES))
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **SWITCHES), check=True,
                         capture_output=True, text=True, timeout=120).stdout
    assert out.strip().endswith("True")
