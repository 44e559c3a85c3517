"""Randomised shape / parameter coverage of the GPU kernels against the oracle
(hypothesis, derandomised so every run checks the same cases).

  * phi^4 step: Lx over every supported row width (one-segment, multi-row and
    multi-segment waves), Ly including partial wave tiles, Lz from 1 (the
    periodic self-neighbour case) upward; C = 0 bit-identical, C = 1 within the
    per-step bound of test_gpu_phi4.py.
  * QM1D serial order: random N, loops, Δτ and potID 0 frames with injected
    reference noise, bit-identical frame by frame.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import PHI4_STEP_ATOL, PHI4_STEP_RTOL, tol_report

pytestmark = pytest.mark.gpu

STEP_ATOL = PHI4_STEP_ATOL   # conftest.py: the measured bound (round 6)
STEP_RTOL = PHI4_STEP_RTOL
FUZZ = settings(max_examples=40, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


@FUZZ
@given(Lx=st.sampled_from([8, 16, 32, 64, 128, 256, 512, 768, 1024]), Ly=st.integers(1, 9),
       Lz=st.integers(1, 12), steps=st.integers(1, 3), C=st.sampled_from([0.0, 1.0]),
       seed=st.integers(0, 2 ** 40), dtau=st.sampled_from([0.005, 0.02, 0.05]))
def test_phi4_random_shapes(gpu, oracle_mod, Lx, Ly, Lz, steps, C, seed, dtau):
    from stochquant_amd import Phi4Lattice
    shape = (Lx, Ly, Lz)
    p = oracle_mod.phi4_params(shape, dtau, 0.5, 1.0, seed, C=C)
    phi = oracle_mod.phi4_init(p, 0.8)
    with Phi4Lattice(shape, dtau=dtau, m2=0.5, lam=1.0, seed=seed, C=C) as L:
        L.upload(phi)
        L.step(steps)
        got = L.download()
    ref = phi
    for s in range(steps):
        ref = oracle_mod.phi4_step(p, ref, s)
    if C == 0.0:
        assert np.array_equal(got, ref)
    else:
        err = np.abs(got.astype(np.float64) - ref)
        tol_report(f"fuzz{shape},dtau={dtau}", err, steps, ref, STEP_RTOL)
        assert np.all(err <= steps * (STEP_ATOL + STEP_RTOL * np.abs(ref)))


def _exact(res):
    for k in ("stable", "dtau", "lrgEl", "lrgVl", "omega", "runs", "seed"):
        assert res[k][0] == res[k][1], (res["frame"], k, res[k])
    for k in ("f", "x", "xx0"):
        assert np.array_equal(res[k][0], res[k][1]), (res["frame"], k)


@settings(max_examples=25, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(N=st.integers(2, 300), loops=st.integers(1, 30), ratio=st.sampled_from([0.05, 0.3, 2.0, 6.0]),
       a=st.sampled_from([0.05, 0.1, 0.5]), seed=st.integers(1, 2 ** 31 - 1))
def test_serial_order_random_frames(gpu, oracle_mod, N, loops, ratio, a, seed):
    from test_gpu_qm1d_serial import _run_pair
    f0 = 0.3 * np.random.default_rng(seed).standard_normal(N)
    _run_pair(oracle_mod, N, a, ratio * a * a, 0, 1.0, loops, seed, 4, f0, check=_exact)


@settings(max_examples=30, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(Lx=st.sampled_from([16, 64, 256, 512]), Ly=st.integers(1, 6), Lz=st.integers(2, 40),
       nslabs=st.integers(2, 8), ghost=st.integers(1, 8), steps=st.integers(1, 20),
       seed=st.integers(0, 2 ** 40))
def test_slab_decomposition_random(gpu, oracle_mod, monkeypatch, Lx, Ly, Lz, nslabs, ghost, steps, seed):
    """T5 as a property: any slab count and ghost depth gives
    the monolithic field bit for bit, noise on."""
    from stochquant_amd import Phi4Lattice
    nslabs = min(nslabs, Lz)
    shape = (Lx, Ly, Lz)
    p = oracle_mod.phi4_params(shape, 0.02, 0.5, 1.0, seed)
    phi = oracle_mod.phi4_init(p, 0.8)
    with Phi4Lattice(shape, dtau=0.02, m2=0.5, lam=1.0, seed=seed) as L:
        L.upload(phi)
        L.step(steps)
        mono = L.download()
    monkeypatch.setenv("SQ_GHOST", str(ghost))
    with Phi4Lattice(shape, dtau=0.02, m2=0.5, lam=1.0, seed=seed, comm="loopback", nslabs=nslabs) as L:
        L.upload(phi)
        L.step(steps)
        assert np.array_equal(L.download(), mono)
