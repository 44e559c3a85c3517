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
    # The multi-process P2P tests fork their rank processes from a fork server
    # started here, before this process makes its first HIP call: a process
    # that has initialised the GPU must never fork+exec (tests/p2p_ranks.py).
    global _FORKSERVER
    if "not gpu" not in config.getoption("markexpr", ""):
        import multiprocessing.forkserver
        multiprocessing.forkserver.ensure_running()
        _FORKSERVER = True


_FORKSERVER = False


def rank_context():
    """multiprocessing context of the P2P rank processes (see pytest_configure)."""
    import multiprocessing
    if not _FORKSERVER:
        pytest.fail("the rank fork server was not started before the first HIP call")
    return multiprocessing.get_context("forkserver")


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
def bm_tables(gpu, sqlib):
    """The device's Box-Muller factors for every 23-bit argument (4 x 2^23
    float32, sq_selftest_bm_tables): with them the oracle's noise is the GPU's
    bit for bit (oracle.device_transcendentals)."""
    import ctypes
    import numpy as np
    t = np.empty(4 << 23, np.float32)
    assert sqlib.sq_selftest_bm_tables(0, t.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 0
    return t


@pytest.fixture
def dev_oracle(oracle_mod, bm_tables):
    """The oracle in device-transcendental mode for the duration of one test."""
    with oracle_mod.device_transcendentals(bm_tables):
        yield oracle_mod


@pytest.fixture(scope="session")
def gpu(sqlib):
    """Skip-free GPU gate: gpu-marked tests must run on a box with a device and fail loudly otherwise."""
    from stochquant_amd import _lib
    n = _lib.device_count()
    if n < 1:
        pytest.fail("no HIP device visible: gpu tests must run on the MI355X box")
    return 0


# fp32 tolerance of a noise-on phi^4 step against the MATHEMATICAL oracle (its
# normals evaluated in double): per step |d| <= PHI4_STEP_ATOL + PHI4_STEP_RTOL
# |phi'|, k steps k x (the update is a contraction for the tested parameters).
# Constants: see tests/test_gpu_phi4.py's header and DESIGN.md §3.
PHI4_STEP_ATOL = 2e-7      # measured need <= 9.6e-8 (profiles/r06/c2/tol.txt)
PHI4_STEP_RTOL = 2.5e-7    # ~2 ulp of |phi'|


def tol_report(name, err, steps, ref, rtol=PHI4_STEP_RTOL, atol=PHI4_STEP_ATOL):
    """Print the measured maximum of a within-tolerance check, the per-step
    absolute term it needs beside `rtol`, and the slack of the bound
    steps * (atol + rtol |ref|) at the worst element (grep 'TOL ' in a -s
    run); return the needed term."""
    import numpy as np
    err = np.asarray(err, dtype=np.float64)
    aref = np.abs(np.asarray(ref, dtype=np.float64))
    need = float(np.max((err - steps * rtol * aref) / steps))
    bound = steps * (atol + rtol * aref)
    nz = err > 0
    slack = float(np.min(bound[nz] / err[nz])) if np.any(nz) else float("inf")
    print(f"TOL {name} max_err={float(err.max()):.4e} steps={steps} atol_needed={need:.4e} "
          f"bound_over_err_min={slack:.2f}", flush=True)
    return need
