"""The resident two-step march (SQ_TB2_RUN=1, csrc/sq_phi4_run.hip): a call's
pairs of steps as ONE launch whose blocks start pair t+1 when their 3 x 3
neighbourhood of blocks has finished pair t.  Bit-identical to one
phi4_tb2_kernel launch per pair (itself bitwise against the oracle,
test_gpu_phi4.py) for every parity of the step count, repeated (a missing or
late hand-off reads a neighbour's plane of the wrong pair in some runs), for
both load forms (an agent-scope acquire per pair, or sc1 loads throughout),
and against the oracle directly; shapes it does not cover fall back to one
launch per pair."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lat(shape, C=1.0, seed=1234, **kw):
    from stochquant_amd import Phi4Lattice
    return Phi4Lattice(shape, dtau=0.02, m2=0.5, lam=1.0, seed=seed, C=C, **kw)


def _field(shape, seed):
    rng = np.random.default_rng(seed)
    return (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)


def _run(monkeypatch, shape, phi0, steps, run, C=1.0, sc1="0", calls=1):
    monkeypatch.setenv("SQ_TB2_RUN", "1" if run else "0")
    monkeypatch.setenv("SQ_TB2_RUN_SC1", sc1)
    with _lat(shape, C=C) as L:
        L.upload(phi0)
        L.perf_reset()
        for _ in range(calls):
            L.step(steps)
        info = L.launch_info()
        out = L.download()
    return out, info


# (shape, steps): 256^3 is the headline lattice (512 blocks, 2 per CU); one
# y-band (every y-neighbour the block itself); a last z-chunk of 2 planes; odd
# step counts (the last step runs as a single-step launch after the march)
CASES = [((256, 256, 256), 20), ((256, 64, 64), 7), ((256, 8, 6), 10), ((256, 16, 40), 41), ((256, 32, 18), 4)]


@pytest.mark.parametrize("sc1", ["0", "1"])
@pytest.mark.parametrize("shape,steps", CASES)
def test_run_kernel_equals_pair_launches(gpu, monkeypatch, shape, steps, sc1):
    phi0 = _field(shape, 5)
    ref, rinfo = _run(monkeypatch, shape, phi0, steps, False)
    assert rinfo["kernel"].startswith("phi4_tb2_kernel<")
    for _ in range(3):
        got, info = _run(monkeypatch, shape, phi0, steps, True, sc1=sc1)
        if steps % 2 == 0:  # (odd: the march and the last single step tie for "launched most")
            assert info["kernel"] == f"phi4_tb2_run_kernel<true, {16 if sc1 == '1' else 0}>", info
            assert info["launches"] == 1
        assert np.array_equal(got, ref)


def test_run_kernel_noiseless_and_calls(gpu, monkeypatch):
    """C = 0 (the NZ = false instance), and several calls in a row: each call's
    epochs continue the previous call's (no clearing between launches)."""
    shape = (256, 32, 32)
    phi0 = _field(shape, 8)
    for C in (0.0, 1.0):
        ref, _ = _run(monkeypatch, shape, phi0, 6, False, C=C, calls=5)
        got, info = _run(monkeypatch, shape, phi0, 6, True, C=C, calls=5)
        assert info["kernel"].startswith(f"phi4_tb2_run_kernel<{'true' if C else 'false'}, ")
        assert info["launches"] == 5
        assert np.array_equal(got, ref)


def test_run_kernel_vs_oracle(gpu, oracle_mod, monkeypatch):
    """Bitwise against the oracle at C = 0, 6 steps (three pairs in one launch)."""
    shape = (256, 16, 8)
    p = oracle_mod.phi4_params(shape, 0.02, 0.5, 1.0, 1234, C=0.0)
    phi0 = oracle_mod.phi4_init(oracle_mod.phi4_params(shape, 0.02, 0.5, 1.0, 77), 0.9)
    ref = phi0
    for s in range(6):
        ref = oracle_mod.phi4_step(p, ref, s)
    got, info = _run(monkeypatch, shape, phi0, 6, True, C=0.0)
    assert info["kernel"] == "phi4_tb2_run_kernel<false, 0>"
    assert np.array_equal(got, ref)


def test_run_kernel_falls_back_on_short_chunks(gpu, monkeypatch):
    """nz = 5: chunks of 4 and 1 planes (the last one's light cone reaches two
    chunks over), so the march does not apply and every pair is its own launch."""
    shape = (256, 8, 5)
    phi0 = _field(shape, 9)
    ref, _ = _run(monkeypatch, shape, phi0, 8, False)
    got, info = _run(monkeypatch, shape, phi0, 8, True)
    assert info["kernel"].startswith("phi4_tb2_kernel<")
    assert np.array_equal(got, ref)
