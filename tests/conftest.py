import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "distributed-correlation_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


import pytest  # noqa: E402


@pytest.fixture
def variant():
    """variant(name, value): an engine implementation switch (dcor_set_variant) for one test,
    restored afterwards.  The engine reads no environment variable."""
    from dcor import _lib
    touched = []

    def set_(name, value):
        touched.append((name, _lib.get_variant(name)))
        _lib.set_variant(name, value)

    yield set_
    for name, old in reversed(touched):
        _lib.set_variant(name, old)
