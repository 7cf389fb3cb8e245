"""The engine build is content-addressed: __graft_entry__.build_engine compares
the sha256 of the engine sources with the hash stamped into libdcor.so and rebuilds on mismatch;
smoke() prints both.  CPU only: no compile here, the decision is checked on a copy of the sources."""
import os
import shutil
import time

import pytest

import __graft_entry__ as g


def test_library_stamp_is_this_trees_sources():
    assert g.stamped_hash() is not None, "libdcor.so carries no source stamp"
    stale, have, want = g.engine_stale()
    assert not stale, f"libdcor.so stamped {have[:16]} but the sources hash to {want[:16]}"


def test_stamp_is_exported_and_matches_bench_hash():
    from bench import src_sha16
    from dcor import _lib
    assert _lib.lib.dcor_source_hash().decode() == g.stamped_hash()
    assert g.source_hash()[:16] == src_sha16()


@pytest.fixture
def tree(tmp_path, monkeypatch):
    """A copy of the engine sources with __graft_entry__ pointed at it."""
    csrc = tmp_path / "distributed-correlation_amd" / "csrc"
    shutil.copytree(g.CSRC, csrc, ignore=shutil.ignore_patterns("*.o"))
    (tmp_path / "include").mkdir()
    shutil.copy(os.path.join(g.ROOT, "include", "dcor.h"), tmp_path / "include" / "dcor.h")
    monkeypatch.setattr(g, "CSRC", str(csrc))
    monkeypatch.setattr(g, "ROOT", str(tmp_path))
    return csrc


def test_touch_without_change_keeps_the_build(tree):
    f = tree / "dcor_fused.hip"
    time.sleep(0.01)
    os.utime(f)   # a newer mtime, same bytes
    assert g.engine_stale()[0] is False


def test_edited_source_triggers_rebuild(tree):
    f = tree / "dcor_premat.hip"
    f.write_text(f.read_text() + "\n// edited\n")
    stale, have, want = g.engine_stale()
    assert stale and have != want and have == g.stamped_hash()


def test_edited_header_triggers_rebuild(tree):
    h = tree.parent.parent / "include" / "dcor.h"
    h.write_text(h.read_text().replace("dcor_version", "dcor_version ", 1))
    assert g.engine_stale()[0]


def test_library_without_stamp_is_stale(tmp_path):
    lib = tmp_path / "libdcor.so"
    lib.write_bytes(b"\x7fELF no stamp here")
    assert g.stamped_hash(str(lib)) is None
    assert g.engine_stale(str(lib))[0]
