import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libstochquant.so)")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: E402  (tests are allowed to use the oracle as the checker)
    oracle.build()
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def sqlib():
    """The product library; built in-tree if missing (hipcc cross-compiles without a GPU)."""
    from stochquant_amd import _lib
    if not os.path.exists(_lib.LIB_PATH) or not os.path.exists(_lib.TAUHOST_PATH):
        from stochquant_amd import build
        build.build()
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(sqlib):
    """Skip-free GPU gate: gpu-marked tests must run on a box with a device and fail loudly otherwise."""
    from stochquant_amd import _lib
    n = _lib.device_count()
    if n < 1:
        pytest.fail("no HIP device visible: gpu tests must run on the MI355X box")
    return 0
