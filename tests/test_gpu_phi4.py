"""3-D φ⁴ hot path on the MI355X vs the oracle.

Parity contract (fp32):
  * C = 0 (noise off): the GPU step is BIT-IDENTICAL to the oracle -- same
    fp32 operations in the same order (explicit fma, -ffp-contract=off).
  * C = 1: the only difference from the mathematical oracle is the hardware
    transcendentals of the noise; one step differs by at most
    sigma*(NORMAL_ATOL + NORMAL_RTOL*|xi|) plus one rounding of phi', i.e.
    |d| <= STEP_ATOL + STEP_RTOL*|phi'|  per step, and the update is a
    contraction for these parameters (row sum of the Jacobian 1 - h*V'' < 1),
    so k steps stay within k times that bound.  With the device's own
    Box-Muller factors (the `dev_oracle` fixture: v_log/v_sqrt/v_cos/v_sin of
    every 23-bit argument, tabulated on the GPU and checked for accuracy in
    test_gpu_selftest.py) the oracle draws the GPU's normals and every C = 1
    result is BIT-IDENTICAL as well (`*_bitwise_device_transcendentals`).
  * Slab decomposition (loopback slabs, RCCL self-exchange) is bit-identical
    to the monolithic run with the noise on.
"""
import ctypes

import numpy as np
import pytest

from conftest import PHI4_STEP_ATOL, PHI4_STEP_RTOL, golden, tol_report

pytestmark = pytest.mark.gpu

# per step |d| <= STEP_ATOL + STEP_RTOL |phi'| against the mathematical oracle
# (k steps: k x): the absolute term covers sigma x the device normals' error
# (measured need <= 9.6e-8 over every within-tolerance test, round 6,
# profiles/r06/c2/tol.txt; round 5's 4e-6 had ~40x slack), the relative one
# ~2 ulp of phi'.  Every check prints its measured maximum (TOL lines, -s).
STEP_ATOL = PHI4_STEP_ATOL
STEP_RTOL = PHI4_STEP_RTOL

SHAPES = [
    (8, 8, 8), (16, 16, 16), (32, 32, 32), (32, 8, 13), (64, 16, 8), (128, 16, 9),
    (256, 8, 8), (256, 4, 33), (512, 4, 4), (768, 2, 5), (1024, 2, 4), (1536, 2, 3),
]


def _lat(shape, C=1.0, dtau=0.02, m2=0.5, lam=1.0, seed=1234, **kw):
    from stochquant_amd import Phi4Lattice
    return Phi4Lattice(shape, dtau=dtau, m2=m2, lam=lam, seed=seed, C=C, **kw)


def _oracle_run(oracle_mod, shape, phi, steps, C=1.0, dtau=0.02, m2=0.5, lam=1.0, seed=1234, step0=0):
    p = oracle_mod.phi4_params(shape, dtau, m2, lam, seed, C=C)
    for s in range(steps):
        phi = oracle_mod.phi4_step(p, phi, step0 + s)
    return phi


def _init(oracle_mod, shape, amp=0.9, seed=77):
    p = oracle_mod.phi4_params(shape, 0.02, 0.5, 1.0, seed)
    return oracle_mod.phi4_init(p, amp)


@pytest.mark.parametrize("shape", SHAPES)
def test_noiseless_step_bitwise(gpu, oracle_mod, shape):
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, C=0.0) as L:
        L.upload(phi0)
        L.step(3)
        got = L.download()
    ref = _oracle_run(oracle_mod, shape, phi0, 3, C=0.0)
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"


@pytest.mark.parametrize("shape", SHAPES)
def test_noisy_step_within_tolerance(gpu, oracle_mod, shape):
    phi0 = _init(oracle_mod, shape)
    k = 4
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(k)
        got = L.download()
    ref = _oracle_run(oracle_mod, shape, phi0, k)
    err = np.abs(got.astype(np.float64) - ref)
    bound = k * (STEP_ATOL + STEP_RTOL * np.abs(ref))
    tol_report(f"phi4_step{shape}", err, k, ref, STEP_RTOL)
    assert np.all(err <= bound)


@pytest.mark.parametrize("shape", SHAPES)
def test_noisy_step_bitwise_device_transcendentals(gpu, dev_oracle, shape):
    phi0 = _init(dev_oracle, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(4)
        got = L.download()
    ref = _oracle_run(dev_oracle, shape, phi0, 4)
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"


@pytest.mark.parametrize("shape,nslabs", [((16, 16, 16), 2), ((32, 8, 13), 3), ((256, 4, 33), 5),
                                          ((64, 16, 8), 8), ((512, 4, 6), 2)])
def test_loopback_decomposition_bitwise(gpu, oracle_mod, shape, nslabs):
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(7)
        mono = L.download()
    with _lat(shape, comm="loopback", nslabs=nslabs) as L:
        L.upload(phi0)
        L.step(7)
        slabs = L.download()
    assert np.array_equal(mono, slabs)


def test_rccl_self_exchange_bitwise(gpu, oracle_mod):
    from stochquant_amd import unique_id
    shape = (64, 16, 12)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(5)
        mono = L.download()
    with _lat(shape, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        L.step(5)
        got = L.download()
    assert np.array_equal(mono, got)


def test_gate_timeout_is_sticky(gpu, oracle_mod, monkeypatch):
    """A gated rim chunk that timed out stores nothing, so the field is corrupt:
    every later sync / download / step / frame fails (not only the first
    report) until a new field is uploaded.  The timeout is flagged through the
    SQ_DIAG_GATE_ERR hook, exactly as tb_gate_wait flags it."""
    from stochquant_amd import StochQuantError, unique_id
    shape = (64, 16, 12)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, loops=4) as L:
        L.upload(phi0)
        L.step(3)
        mono = L.download()
    with _lat(shape, loops=4, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        monkeypatch.setenv("SQ_DIAG_GATE_ERR", "1")
        L.step(1)
        monkeypatch.delenv("SQ_DIAG_GATE_ERR")
        for call in (L.sync, L.sync, L.download, lambda: L.step(1), L.run_frame, L.sync):
            with pytest.raises(StochQuantError, match="gated rim chunks timed out"):
                call()
        L.upload(phi0)  # a new field clears it
        L.step_counter = 0
        L.step(3)
        L.sync()
        assert np.array_equal(L.download(), mono)


def test_full_size_256_one_step(gpu, oracle_mod, bm_tables):
    """BASELINE config C2 (256^3 fp32): one step vs the oracle (within the
    tolerance of the mathematical normals, bitwise with the device's), and the
    decomposition invariance at full size."""
    shape = (256, 256, 256)
    phi0 = _init(oracle_mod, shape, amp=0.5)
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0) as L:
        L.upload(phi0)
        L.step(1)
        got = L.download()
    ref = _oracle_run(oracle_mod, shape, phi0, 1, dtau=0.01, m2=1.0, lam=1.0)
    err = np.abs(got.astype(np.float64) - ref)
    tol_report("full_size_256_one_step", err, 1, ref, STEP_RTOL)
    assert np.all(err <= STEP_ATOL + STEP_RTOL * np.abs(ref))
    with oracle_mod.device_transcendentals(bm_tables):
        assert np.array_equal(got, _oracle_run(oracle_mod, shape, phi0, 1, dtau=0.01, m2=1.0, lam=1.0))
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, comm="loopback", nslabs=4) as L:
        L.upload(phi0)
        L.step(1)
        assert np.array_equal(L.download(), got)


def test_guard_clamp_nan_and_rollback(gpu, oracle_mod):
    shape = (32, 8, 8)
    phi0 = _init(oracle_mod, shape, amp=0.3)
    phi0[3, 4, 5] = np.float32(5e3)
    phi0[6, 1, 30] = np.float32("nan")
    with _lat(shape, C=0.0, loops=3) as L:
        L.upload(phi0)
        L.step(1)
        got = L.download()
    ref = _oracle_run(oracle_mod, shape, phi0, 1, C=0.0)
    assert np.array_equal(got, ref)
    assert np.all(np.abs(got) <= 1000)
    with _lat(shape, loops=3) as L:
        L.upload(phi0)
        d0 = L.dtau
        stable = L.run_frame()
        assert not stable
        back = L.download()
        assert np.array_equal(back[~np.isnan(phi0)], phi0[~np.isnan(phi0)])
        assert np.isnan(back[6, 1, 30])
        assert L.dtau == pytest.approx(d0 * 0.95)
        assert L.step_counter == 3      # retried frames draw fresh noise


def test_stable_frames_grow_dtau(gpu, oracle_mod):
    shape = (16, 16, 16)
    with _lat(shape, loops=5, dtau=0.01) as L:
        L.init_field(0.2)
        d0 = L.dtau
        for _ in range(12):
            assert L.run_frame()
        assert L.dtau == pytest.approx(d0 / 0.95)  # tauhost.c:523-528: after 11 stable frames


def test_init_field_matches_oracle(gpu, oracle_mod, bm_tables):
    shape = (64, 16, 8)
    with _lat(shape, seed=77) as L:
        L.init_field(0.9)
        got = L.download()
    ref = _init(oracle_mod, shape, amp=0.9, seed=77)
    assert np.all(np.abs(got - ref) <= 0.9 * (2e-6 + 2e-6 * np.abs(ref / 0.9)))
    with oracle_mod.device_transcendentals(bm_tables):
        assert np.array_equal(got, _init(oracle_mod, shape, amp=0.9, seed=77))


def test_moments_and_correlator(gpu, oracle_mod):
    shape = (32, 16, 24)
    with _lat(shape) as L:
        L.init_field(0.7)
        L.step(3)
        phi = L.download().astype(np.float64)
        m = L.moments()
        c = L.correlator(6)
    assert m["sum"] == pytest.approx(phi.sum(), rel=1e-9, abs=1e-9)
    assert m["sum2"] == pytest.approx((phi ** 2).sum(), rel=1e-9)
    assert m["maxabs"] == np.abs(phi).max()
    S = phi.sum(axis=(1, 2))
    ref = np.array([np.sum(S * np.roll(S, -t)) for t in range(6)]) / phi.size
    assert np.allclose(c, ref, rtol=1e-9)


def test_free_field_variance_kat(gpu):
    """lambda = 0: <phi^2> relaxes to the exact Euler-Maruyama value
    mean_k [lam_k (1 - h lam_k/2)]^-1 (tests/golden/analytic_kats.json)."""
    g = golden("analytic_kats.json")["free_var_3d_L32"]
    L0 = g["L"]
    with _lat((L0, L0, L0), dtau=g["h"], m2=g["m2"], lam=0.0, seed=4321) as L:
        L.init_field(0.0)
        L.step(500)
        samples = []
        for _ in range(200):
            L.step(10)
            samples.append(L.moments()["sum2"] / L0 ** 3)
    s = np.array(samples)
    blocks = s.reshape(20, 10).mean(axis=1)     # blocks of 100 steps ~ 1 autocorrelation time
    err = blocks.std(ddof=1) / np.sqrt(len(blocks))
    print("free var", s.mean(), "+-", err, "exact", g["value"])
    assert abs(s.mean() - g["value"]) < 4 * err + 5e-4


def test_unsupported_shape_fails_loudly(gpu):
    from stochquant_amd import StochQuantError
    with pytest.raises(StochQuantError):
        _lat((20, 8, 8))


@pytest.mark.parametrize("ghost,nslabs,steps", [(1, 2, 5), (2, 3, 7), (4, 2, 9), (4, 4, 8), (8, 2, 13), (3, 5, 4)])
def test_deep_halo_blocks_bitwise(gpu, oracle_mod, monkeypatch, ghost, nslabs, steps):
    """Ghost-zone depth G: one exchange per G steps, ghost sites recomputed
    redundantly; partial blocks when steps % G != 0.  Bit-identical to the
    single-slab run (counter-based noise makes redundant sites exact)."""
    shape = (32, 16, 24)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(steps)
        mono = L.download()
    monkeypatch.setenv("SQ_GHOST", str(ghost))
    with _lat(shape, comm="loopback", nslabs=nslabs) as L:
        L.upload(phi0)
        for n in (1, steps - 1):
            L.step(n)
        assert np.array_equal(mono, L.download())


def test_rccl_self_exchange_deep_halo_frames(gpu, oracle_mod, monkeypatch):
    from stochquant_amd import unique_id
    shape = (256, 8, 16)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, loops=6) as L:
        L.upload(phi0)
        for _ in range(3):
            assert L.run_frame()
        mono = L.download()
    monkeypatch.setenv("SQ_GHOST", "4")
    with _lat(shape, loops=6, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        for _ in range(3):
            assert L.run_frame()
        assert np.array_equal(mono, L.download())


@pytest.mark.parametrize("shape", [(256, 8, 8), (256, 4, 33), (512, 4, 6), (256, 16, 5)])
@pytest.mark.parametrize("pf", [1, 3, 4, 7])
def test_prefetch_variants_bitwise(gpu, oracle_mod, monkeypatch, shape, pf):
    monkeypatch.setenv("SQ_PREFETCH", str(pf))
    monkeypatch.setenv("SQ_FUSE2", "0")  # every step through the per-step kernel variant
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, C=0.0) as L:
        L.upload(phi0)
        L.step(3)
        got = L.download()
    assert np.array_equal(got, _oracle_run(oracle_mod, shape, phi0, 3, C=0.0))


def _full_size_check(oracle_mod, shape, steps, tables=None, **kw):
    """`steps` steps of the lattice context built with **kw, C = 0 (bitwise) and
    C = 1 vs the oracle -- bitwise with the device's Box-Muller factors
    (`tables`), else within the per-step tolerance -- returning the C = 1 field."""
    from stochquant_amd import unique_id
    phi0 = _init(oracle_mod, shape, amp=0.5)
    out = None
    for C in (0.0, 1.0):
        if kw.get("comm") == "rccl":   # a fresh RCCL unique id per communicator
            kw = dict(kw, nranks=1, rank=0, comm_id=unique_id())
        with _lat(shape, C=C, dtau=0.01, m2=1.0, lam=1.0, **kw) as L:
            L.upload(phi0)
            L.step(steps)
            got = L.download()
            kname = L.kernel_name
        if C == 1.0 and tables is not None:
            with oracle_mod.device_transcendentals(tables):
                ref = _oracle_run(oracle_mod, shape, phi0, steps, C=C, dtau=0.01, m2=1.0, lam=1.0)
            assert np.array_equal(got, ref), f"{kname} (C = 1): max diff {np.max(np.abs(got - ref))}"
            out = got
            del got, ref
            continue
        ref = _oracle_run(oracle_mod, shape, phi0, steps, C=C, dtau=0.01, m2=1.0, lam=1.0)
        if C == 0.0:
            assert np.array_equal(got, ref), f"{kname}: max diff {np.max(np.abs(got - ref))}"
        else:
            err = np.abs(got.astype(np.float64) - ref)
            tol_report(f"full_size{shape}{kw}", err, steps, ref, STEP_RTOL)
            assert np.all(err <= steps * (STEP_ATOL + STEP_RTOL * np.abs(ref))), f"{kname}: max err {err.max()}"
            out = got
        del got, ref
    return phi0, out


def test_full_size_512(gpu, oracle_mod, bm_tables):
    """BASELINE config C3 (512^3 fp32, 2 x 512 MiB, the HBM-bound case): two
    steps (one launch pair of whatever the library runs at 512^3) vs the
    oracle, bitwise at C = 0 and (device Box-Muller factors) at C = 1."""
    _full_size_check(oracle_mod, (512, 512, 512), 2, tables=bm_tables)


@pytest.mark.parametrize("ghost", ["16", "auto"])
def test_c5_slab_1024x1024x128_rccl(gpu, oracle_mod, bm_tables, monkeypatch, ghost):
    """BASELINE config C5's per-GPU slab (1024^3 over 8 GPUs = 1024 x 1024 x 128
    planes per rank) through the RCCL slab path (self-exchange: the same
    deep-halo blocks, exchange and stream joins as a multi-rank run), G = 16
    and the timed ghost-depth trial: one step vs the oracle (bitwise at C = 0),
    and 100 steps (trial blocks + fused pairs) bit-identical to the single-slab run."""
    from stochquant_amd import unique_id
    shape = (1024, 1024, 128)
    if ghost == "auto":
        monkeypatch.setenv("SQ_GHOST_AUTO", "1")
    else:
        monkeypatch.setenv("SQ_GHOST", ghost)
    phi0, _ = _full_size_check(oracle_mod, shape, 1, tables=bm_tables, comm="rccl")
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0) as L:
        L.upload(phi0)
        L.step(100)
        mono = L.download()
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        L.step(100)
        act, alloc = L.ghost
        assert act == 16 if ghost == "16" else act in (4, 8, 16)
        assert np.array_equal(L.download(), mono)


def test_full_size_256_rccl_slab_fused_vs_oracle(gpu, oracle_mod, bm_tables, monkeypatch):
    """C2/C4's per-GPU slab through the RCCL slab path with the inner steps of
    each block fused in pairs (G = 4: core/rim step 0, a pair, the edges-first
    last step): 4 steps vs the oracle -- bitwise at C = 0 and, with the
    device's Box-Muller factors, at C = 1."""
    monkeypatch.setenv("SQ_GHOST", "4")
    monkeypatch.setenv("SQ_FUSE2", "1")
    _full_size_check(oracle_mod, (256, 256, 256), 4, tables=bm_tables, comm="rccl")


FUSE2_SHAPES = [(256, 8, 2), (256, 8, 5), (256, 16, 12), (256, 32, 33), (256, 64, 64), (256, 24, 17),
                # rows of several 256-site segments: the x-halo wave supplies the segment-edge sites
                (512, 8, 5), (512, 16, 12), (768, 8, 7), (1024, 8, 9), (512, 24, 17)]


@pytest.mark.parametrize("shape", FUSE2_SHAPES)
@pytest.mark.parametrize("zb", [1, 3, 16])
@pytest.mark.parametrize("C", [0.0, 1.0])
@pytest.mark.parametrize("wpe", ["6", "1"])
def test_fused_two_step_bitwise(gpu, oracle_mod, monkeypatch, shape, zb, C, wpe):
    """Steps s and s+1 in one launch (8-row y-bands with their halo rows and
    the chunk-edge planes of step s recomputed per block) == two single-step
    launches, bit for bit; odd step counts end with one single step."""
    phi0 = _init(oracle_mod, shape)
    monkeypatch.setenv("SQ_FUSE2", "0")
    with _lat(shape, C=C) as L:
        L.upload(phi0)
        L.step(9)
        ref = L.download()
    if wpe == "1" and shape[0] == 256:
        pytest.skip("the register-budget variant exists for rows of several segments only")
    monkeypatch.setenv("SQ_FUSE2", "1")
    monkeypatch.setenv("SQ_FUSE2_Z", str(zb))
    monkeypatch.setenv("SQ_TB2_WPE", wpe)
    with _lat(shape, C=C) as L:
        assert "tb2" in L.kernel_name, L.kernel_name
        L.upload(phi0)
        for n in (1, 4, 3, 1):
            L.step(n)
        got = L.download()
        assert L.step_counter == 9
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"
    if C == 0.0:
        assert np.array_equal(got, _oracle_run(oracle_mod, shape, phi0, 9, C=0.0))


@pytest.mark.parametrize("shape,ghost,nslabs,steps", [((256, 8, 24), 2, 2, 7), ((256, 8, 24), 4, 3, 13),
                                                      ((256, 16, 40), 5, 3, 11), ((256, 16, 40), 8, 2, 17),
                                                      ((256, 8, 30), 3, 4, 9), ((512, 8, 24), 4, 2, 13),
                                                      ((1024, 8, 30), 5, 3, 11)])
def test_fused_two_step_deep_halo_bitwise(gpu, oracle_mod, monkeypatch, shape, ghost, nslabs, steps):
    """Deep-halo blocks with the inner steps fused in pairs (the pair writes the
    second step's shrinking ghost range) == the single-slab run with one step
    per launch, bit for bit, over several blocks and a partial one."""
    phi0 = _init(oracle_mod, shape)
    monkeypatch.setenv("SQ_FUSE2", "0")
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(steps)
        mono = L.download()
    monkeypatch.setenv("SQ_FUSE2", "1")
    monkeypatch.setenv("SQ_FUSE2_Z", "3")
    monkeypatch.setenv("SQ_GHOST", str(ghost))
    with _lat(shape, comm="loopback", nslabs=nslabs) as L:
        assert "tb2" in L.kernel_name
        L.upload(phi0)
        for n in (1, steps - 1):
            L.step(n)
        assert np.array_equal(mono, L.download())


@pytest.mark.parametrize("core_pairs,rims_b,gate,stopev", [("0", "0", "0", "0"), ("1", "0", "0", "0"), ("1", "0", "1", "0"),
                                                            ("1", "0", "0", "1"), ("0", "0", "0", "1"),
                                                            ("1", "1", "0", "0"), ("2", "0", "0", "0"),
                                                            ("2", "1", "0", "0"), ("4", "0", "0", "0"),
                                                            ("4", "1", "0", "1"), ("8", "1", "0", "0")])
def test_core_pairs_ahead_of_the_exchange_bitwise(gpu, oracle_mod, monkeypatch, core_pairs, rims_b, gate, stopev):
    """K fused core pairs before the exchange wait (K = 0: none, the first
    pair waits for the exchange), their rims after it on stream A or on the
    exchange stream (the C4 overlap for slow links), K = 1 also as the gated
    launch (SQ_SLAB_GATE=1: rim chunks wait in-kernel for the exchange): RCCL
    self-exchange, P2P self-exchange and loopback slabs == the single-slab
    run, bit for bit, over full and partial blocks; EDGES_DONE as a marker or
    as the stop event of the pair before it (SQ_EDGES_STOPEV)."""
    monkeypatch.setenv("SQ_SLAB_GATE", gate)
    monkeypatch.setenv("SQ_EDGES_STOPEV", stopev)
    from stochquant_amd import unique_id
    shape = (256, 16, 96)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(37)
        mono = L.download()
    monkeypatch.setenv("SQ_CORE_PAIRS", core_pairs)
    monkeypatch.setenv("SQ_RIMS_B", rims_b)
    monkeypatch.setenv("SQ_GHOST", "16")
    monkeypatch.setenv("SQ_FUSE2", "1")
    for kw in (dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id()), dict(comm="loopback", nslabs=2),
               dict(comm="p2p", nranks=1, rank=0)):
        with _lat(shape, **kw) as L:
            if kw["comm"] == "p2p":
                L.p2p_connect([L.p2p_handle()])
            L.upload(phi0)
            for n in (16, 21):
                L.step(n)
            assert np.array_equal(L.download(), mono), kw["comm"]


@pytest.mark.parametrize("ghost", ["4", "16"])
@pytest.mark.parametrize("kstage", ["0", "1"])
def test_exchange_on_interior_stream_bitwise(gpu, oracle_mod, monkeypatch, ghost, kstage):
    """SQ_XCHG_ON_A=1: the exchange (RCCL send / recv; P2P staging, hand-shake
    and pull, the staging slot written by the last pair under SQ_P2P_KSTAGE=1)
    runs in order on the interior stream between a block's last pair and the
    next block's first: RCCL and P2P self-exchange == the single slab, bit for
    bit, over full and partial blocks and a frame in between."""
    from stochquant_amd import unique_id
    shape = (256, 16, 96)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, loops=6) as L:
        L.upload(phi0)
        L.step(16)
        L.step(21)
        ok = L.run_frame()
        L.step(9)
        mono = L.download()
    monkeypatch.setenv("SQ_XCHG_ON_A", "1")
    monkeypatch.setenv("SQ_P2P_KSTAGE", kstage)
    monkeypatch.setenv("SQ_GHOST", ghost)
    monkeypatch.setenv("SQ_FUSE2", "1")
    for kw in (dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id()), dict(comm="p2p", nranks=1, rank=0)):
        with _lat(shape, loops=6, **kw) as L:
            if kw["comm"] == "p2p":
                L.p2p_connect([L.p2p_handle()])
            assert L.schedule["core_pairs"] == 0
            L.upload(phi0)
            L.step(16)
            L.step(21)
            assert L.run_frame() == ok
            L.step(9)
            assert np.array_equal(L.download(), mono), kw["comm"]


def test_fused_two_step_rccl_frames(gpu, oracle_mod, monkeypatch):
    """RCCL self-exchange slab with fused inner steps, run as frames."""
    from stochquant_amd import unique_id
    shape = (256, 16, 32)
    phi0 = _init(oracle_mod, shape)
    monkeypatch.setenv("SQ_FUSE2", "0")
    with _lat(shape, loops=7) as L:
        L.upload(phi0)
        for _ in range(3):
            assert L.run_frame()
        mono = L.download()
    monkeypatch.setenv("SQ_FUSE2", "1")
    monkeypatch.setenv("SQ_GHOST", "6")
    with _lat(shape, loops=7, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        for _ in range(3):
            assert L.run_frame()
        assert np.array_equal(mono, L.download())


def test_fused_two_step_full_size_256(gpu, oracle_mod, monkeypatch):
    """C2 at full size: 40 steps as 20 fused launches == 40 single steps."""
    shape = (256, 256, 256)
    phi0 = _init(oracle_mod, shape, amp=0.5)
    outs = []
    for fz in ("0", "1"):
        monkeypatch.setenv("SQ_FUSE2", fz)
        with _lat(shape, dtau=0.01, m2=1.0, lam=1.0) as L:
            assert ("tb2" in L.kernel_name) == (fz == "1")
            L.upload(phi0)
            L.step(40)
            outs.append(L.download())
    assert np.array_equal(outs[0], outs[1])


def test_fused_two_step_guard_and_rollback(gpu, oracle_mod, monkeypatch):
    """A clamp / NaN in either fused step raises the frame's guard flag."""
    monkeypatch.setenv("SQ_FUSE2", "1")
    shape = (256, 8, 8)
    phi0 = _init(oracle_mod, shape, amp=0.3)
    phi0[3, 4, 5] = np.float32(5e3)
    phi0[6, 1, 130] = np.float32("nan")
    with _lat(shape, C=0.0, loops=4) as L:
        assert "tb2" in L.kernel_name
        L.upload(phi0)
        L.step(2)
        assert np.array_equal(L.download(), _oracle_run(oracle_mod, shape, phi0, 2, C=0.0))
    with _lat(shape, loops=4) as L:
        L.upload(phi0)
        assert not L.run_frame()
        back = L.download()
        assert np.array_equal(back[~np.isnan(phi0)], phi0[~np.isnan(phi0)])
    phi1 = _init(oracle_mod, shape, amp=0.3)
    with _lat(shape, loops=4) as L:
        L.upload(phi1)
        assert L.run_frame()


@pytest.mark.parametrize("shape", [(512, 4, 6), (1024, 2, 5), (512, 8, 9)])
@pytest.mark.parametrize("vseg", [1, 2])
def test_segments_per_lane_bitwise(gpu, oracle_mod, monkeypatch, shape, vseg):
    """V float4 segments per lane (x = 256 v + 4 lane) vs separate waves per
    256-site segment with edge loads: both bit-identical to the oracle."""
    monkeypatch.setenv("SQ_VSEG", str(vseg))
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, C=0.0) as L:
        assert L.tile[3] == vseg
        L.upload(phi0)
        L.step(3)
        got = L.download()
    assert np.array_equal(got, _oracle_run(oracle_mod, shape, phi0, 3, C=0.0))


def test_checkpoint_roundtrip_resumes_noise_bitwise(gpu, oracle_mod, tmp_path):
    """Binary checkpoint (sq_save_field / sq_load_field): save after k steps,
    load into a fresh context, continue m steps == the uninterrupted k+m run,
    bit for bit (the Philox step counter and Δτ travel in <path>.json)."""
    import json
    shape = (64, 16, 12)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, loops=4) as L:
        L.upload(phi0)
        assert L.run_frame()
        L.save(tmp_path / "ck.npy")
        saved = L.download()
        L.step(6)
        full = L.download()
        d_full = L.dtau
    assert np.array_equal(np.load(tmp_path / "ck.npy"), saved)
    meta = json.loads((tmp_path / "ck.npy.json").read_text())
    assert meta["dims"] == [64, 16, 12] and meta["step"] == 4 and meta["seed"] == 1234
    with _lat(shape, loops=4, dtau=0.5) as L:
        L.load(tmp_path / "ck.npy")
        assert L.step_counter == 4 and L.dtau == d_full
        L.step(6)
        assert np.array_equal(L.download(), full)
    with _lat((64, 16, 13)) as L:
        from stochquant_amd import StochQuantError
        with pytest.raises(StochQuantError):
            L.load(tmp_path / "ck.npy")


def test_checkpoint_large_seed_and_frame_state(gpu, oracle_mod, tmp_path):
    """Seeds >= 2^63 round-trip through the checkpoint metadata (unsigned
    parse), and a resume carries the frame state across: the stability
    heuristic's T and V and the dtau controller's stable-frame count, so
    frames after the load equal the uninterrupted run's (field, dtau, T, V)."""
    import json
    shape, seed = (256, 8, 12), 0xFEDCBA9876543210
    phi0 = _init(oracle_mod, shape, amp=0.3)
    with _lat(shape, loops=4, seed=seed, dtau=0.01) as L:
        L.upload(phi0)
        for _ in range(7):
            assert L.run_frame()
        L.save(tmp_path / "ck.npy")
        st0 = L.stability()
        for _ in range(9):                  # crosses the 11-stable-frames dtau growth
            assert L.run_frame()
        full, d_full, st_full = L.download(), L.dtau, L.stability()
    meta = json.loads((tmp_path / "ck.npy.json").read_text())
    assert meta["seed"] == seed and meta["stab_cnt"] == 7 and meta["stab_init"] == 1
    assert np.float32(meta["stab_T"]) == np.float32(st0["T"]) and np.float32(meta["stab_V"]) == np.float32(st0["V"])
    with _lat(shape, loops=4, seed=seed, dtau=0.01) as L:
        L.load(tmp_path / "ck.npy")
        st = L.stability(0)
        assert st["T"] == st0["T"] and st["V"] == st0["V"]
        for _ in range(9):
            assert L.run_frame()
        assert L.dtau == d_full and d_full > 0.01
        st = L.stability()
        assert st["T"] == st_full["T"] and st["V"] == st_full["V"]
        assert np.array_equal(L.download(), full)


def test_checkpoint_non_finite_frame_state_is_valid_json(gpu, oracle_mod, tmp_path):
    """a frame on an uploaded field holding inf seeds V = inf (the
    field's max |phi|); the checkpoint metadata must stay valid JSON (T / V as
    null, their exact IEEE bits beside them) and a load must restore T and V
    bit for bit."""
    import json
    shape = (256, 8, 12)
    phi0 = _init(oracle_mod, shape, amp=0.3)
    phi0[3, 2, 17] = np.inf
    with _lat(shape, loops=4, dtau=0.01) as L:
        L.upload(phi0)
        L.run_frame()                     # the guard clamps the inf: rolled back, V seeded inf
        st0 = L.stability(0)
        assert not np.isfinite(st0["V"])
        L.save(tmp_path / "ck.npy")
    meta = json.loads((tmp_path / "ck.npy.json").read_text())   # strict JSON: no bare inf / nan
    assert meta["stab_V"] is None
    assert np.array([meta["stab_V_bits"]], np.uint32).view(np.float32)[0] == np.float32(st0["V"])
    assert np.array([meta["stab_T_bits"]], np.uint32).view(np.float32)[0].tobytes() == \
        np.float32(st0["T"]).tobytes()
    with _lat(shape, loops=4, dtau=0.01) as L:
        L.load(tmp_path / "ck.npy")
        st = L.stability(0)
        assert np.float32(st["V"]).tobytes() == np.float32(st0["V"]).tobytes()
        assert np.float32(st["T"]).tobytes() == np.float32(st0["T"]).tobytes()


def test_slice_correlator_across_slabs(gpu, oracle_mod):
    """The zero-momentum correlator of a decomposed lattice (loopback slabs;
    RCCL self-exchange = the all-reduce code path of the multi-rank case) equals
    the single-slab one exactly: per-plane sums are the same kernels."""
    from stochquant_amd import unique_id
    shape = (64, 16, 24)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(3)
        mono = L.correlator(24)
    with _lat(shape, comm="loopback", nslabs=3) as L:
        L.upload(phi0)
        L.step(3)
        assert np.array_equal(L.correlator(24), mono)
    with _lat(shape, comm="rccl", nranks=1, rank=0, comm_id=unique_id()) as L:
        L.upload(phi0)
        L.step(3)
        assert np.array_equal(L.correlator(24), mono)


@pytest.mark.parametrize("comm", ["loopback", "rccl", "rccl_overlap"])
def test_ghost_autotune_is_exact(gpu, oracle_mod, monkeypatch, comm):
    """Timed trial blocks pick G in {4, 8, 16} and the core pairs that run
    ahead of the exchange in {1, 2, 4} (rccl_overlap: the exchange pinned to
    its own stream; rccl: one rank's default, the exchange in order on the
    interior stream); the trial steps are ordinary steps, so the field after
    them equals the single-slab run bit for bit."""
    from stochquant_amd import unique_id
    monkeypatch.setenv("SQ_GHOST_AUTO", "1")
    if comm == "rccl_overlap":
        monkeypatch.setenv("SQ_XCHG_ON_A", "0")
    shape = (256, 8, 128)
    phi0 = _init(oracle_mod, shape)
    steps = 390            # >= 3*(4+8+16) + 6*3*16 = 372 trial steps, then 18 more
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(steps)
        mono = L.download()
    kw = dict(comm="loopback", nslabs=2) if comm == "loopback" else \
        dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id())
    with _lat(shape, **kw) as L:
        L.upload(phi0)
        L.step(steps)
        act, alloc = L.ghost
        assert alloc == 16 and act in (4, 8, 16)
        sch = L.schedule
        assert sch["tuned"] and sch["core_pairs"] in (0, 1, 2, 4) and sch["edge_first"] in (False, True)
        assert L.step_counter == steps
        assert np.array_equal(L.download(), mono)


def test_uneven_slabs_edge_first(gpu, oracle_mod, monkeypatch):
    """Slabs of different thickness in one decomposition: only the thicker ones
    split their last step into edges + middle; each slab's exchange must wait on
    its own edge event (regression: Lz = 31 over 5 slabs, G = 3)."""
    shape = (16, 4, 31)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape) as L:
        L.upload(phi0)
        L.step(10)
        mono = L.download()
    monkeypatch.setenv("SQ_GHOST", "3")
    with _lat(shape, comm="loopback", nslabs=5) as L:
        L.upload(phi0)
        L.step(4)
        L.step(6)
        assert np.array_equal(L.download(), mono)


def test_checkpoint_load_validates_before_touching_the_field(gpu, oracle_mod, tmp_path):
    """sq_load_field checks the .npy header against the slab before allocating,
    and the metadata's dims / z0 / seed before uploading: every bad checkpoint
    fails with an error and leaves the context's field and counters as they were."""
    import json
    from stochquant_amd import StochQuantError
    shape = (64, 16, 12)
    phi0 = _init(oracle_mod, shape)
    with _lat(shape, seed=1234) as L:
        L.upload(phi0)
        L.step(2)
        L.save(tmp_path / "ck.npy")
    meta = json.loads((tmp_path / "ck.npy.json").read_text())
    bad = {}
    m = dict(meta, seed=999)
    bad["seed"] = m
    m = dict(meta, dims=[64, 16, 13])
    bad["dims"] = m
    m = dict(meta, z0=5)
    bad["z0"] = m
    for name, m in bad.items():
        d = tmp_path / name
        d.mkdir()
        (d / "ck.npy").write_bytes((tmp_path / "ck.npy").read_bytes())
        (d / "ck.npy.json").write_text(json.dumps(m))
    # a header claiming a huge shape (would have allocated terabytes before the check)
    raw = bytearray((tmp_path / "ck.npy").read_bytes())
    hdr = raw[10:10 + (raw[8] | raw[9] << 8)].decode()
    hdr2 = hdr.replace("'shape': (12, 16, 64)", "'shape': (99999999, 99999, 64)")
    hdr2 = hdr2[:len(hdr)] if len(hdr2) >= len(hdr) else hdr2 + " " * (len(hdr) - len(hdr2))
    d = tmp_path / "huge"
    d.mkdir()
    (d / "ck.npy").write_bytes(bytes(raw[:10]) + hdr2.encode() + bytes(raw[10 + len(hdr):]))
    (d / "ck.npy.json").write_text(json.dumps(meta))
    with _lat(shape, seed=1234) as L:
        L.upload(phi0)
        L.step_counter = 7
        for name in list(bad) + ["huge"]:
            with pytest.raises(StochQuantError):
                L.load(tmp_path / name / "ck.npy")
            assert np.array_equal(L.download(), phi0), name
            assert L.step_counter == 7
        L.load(tmp_path / "seed" / "ck.npy", restore_counters=False)   # a field as an initial condition
        assert L.step_counter == 7


STAB_CASES = [((256, 8, 8), {}), ((64, 16, 8), {}), ((512, 8, 6), {"SQ_FUSE2": "1"}),
              ((256, 8, 12), {"comm": "loopback", "nslabs": 3}), ((256, 16, 16), {"comm": "rccl"})]


@pytest.mark.parametrize("shape,opt", STAB_CASES)
def test_stability_rule_rolls_back_diverging_unclamped_field(gpu, oracle_mod, monkeypatch, shape, opt):
    """The reference's stability heuristic (tau_kernel.cl:135-143) restated for
    the 3-D lattice: Euler at dtau = 0.2 > 2/lambda_max diverges
    as an oscillation that stays far below the clamp within the frame, so only
    the heuristic can catch it.  Per-step records (M, D, A), the firing step,
    the carried T / V and the rollback are bit-identical to the oracle's
    statement of the same rule (C = 0), through the fused, per-step,
    multi-segment, loopback-slab and RCCL-slab paths."""
    from stochquant_amd import unique_id
    kw = dict(opt)
    for k in [k for k in kw if k.startswith("SQ_")]:
        monkeypatch.setenv(k, kw.pop(k))
    if kw.get("comm") == "rccl":
        kw.update(nranks=1, rank=0, comm_id=unique_id())
        monkeypatch.setenv("SQ_GHOST", "4")
    loops, h = 12, 0.2
    phi0 = _init(oracle_mod, shape, amp=0.05)
    p = oracle_mod.phi4_params(shape, h, 1.0, 1.0, 1234, C=0.0)
    T0, V0 = float(phi0.max()), float(np.abs(phi0).max())
    out, M, D, A, fired, T1, V1 = oracle_mod.phi4_frame_stab(p, phi0, loops, 0, T0, V0)
    assert fired >= 0 and np.abs(out).max() < 1000        # diverging, never clamped
    with _lat(shape, C=0.0, dtau=h, m2=1.0, lam=1.0, loops=loops, **kw) as L:
        L.upload(phi0)
        assert not L.run_frame()
        st = L.stability()
        assert np.array_equal(st["M"], M) and np.array_equal(st["D"], D) and np.array_equal(st["A"], A)
        assert st["fired"] == fired and st["T"] == T1 and st["V"] == V1
        assert np.array_equal(L.download(), phi0)           # rolled back
        assert L.dtau == pytest.approx(h * 0.95)
        assert L.step_counter == loops                      # a retried frame draws fresh noise


def test_stability_rule_quiet_on_stable_frames(gpu, oracle_mod, bm_tables):
    """dtau = 0.01, noise on: the heuristic never fires, records within the
    noise tolerance of the mathematical oracle's and identical to the
    oracle's with the device's Box-Muller factors."""
    shape, loops = (256, 16, 16), 6
    phi0 = _init(oracle_mod, shape, amp=0.3)
    p = oracle_mod.phi4_params(shape, 0.01, 1.0, 1.0, 1234, C=1.0)
    out, M, D, A, fired, T1, V1 = oracle_mod.phi4_frame_stab(p, phi0, loops, 0, float(phi0.max()),
                                                            float(np.abs(phi0).max()))
    assert fired == -1
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, loops=loops) as L:
        L.upload(phi0)
        assert L.run_frame()
        st = L.stability()
        assert st["fired"] == -1
        got = L.download()
        for nm, g_, r_ in (("M", st["M"], M), ("A", st["A"], A), ("D", st["D"], D), ("field", got, out)):
            r64 = np.asarray(r_, np.float64)
            e = np.abs(np.asarray(g_, np.float64) - r64)
            tol_report(f"stab_records_{nm}", e, loops, r64, STEP_RTOL)
            assert np.all(e <= loops * (STEP_ATOL + STEP_RTOL * np.abs(r64))), (nm, float(e.max()))
    # the device's Box-Muller factors: records, T, V and the field bit for bit
    with oracle_mod.device_transcendentals(bm_tables):
        out, M, D, A, fired, T1, V1 = oracle_mod.phi4_frame_stab(p, phi0, loops, 0, float(phi0.max()),
                                                                float(np.abs(phi0).max()))
    assert fired == -1
    assert np.array_equal(st["M"], M) and np.array_equal(st["D"], D) and np.array_equal(st["A"], A)
    assert st["T"] == T1 and st["V"] == V1
    assert np.array_equal(got, out)


@pytest.mark.parametrize("shape", [(256, 16, 12), (512, 8, 9)])
@pytest.mark.parametrize("loops", [2, 3, 5])
def test_frame_snapshot_from_first_fused_launch(gpu, oracle_mod, shape, loops):
    """A one-stream frame's rollback snapshot is stored by its first fused
    launch (Phi4StepArgs::snap): after stable frames have moved
    the field between the ping-pong buffers, an unstable frame (a clamp hit
    and a NaN) still restores the frame-start field bit for bit, odd frame
    lengths (a fused pair, then per-step launches) included."""
    phi0 = _init(oracle_mod, shape, amp=0.3)
    with _lat(shape, loops=loops) as L:
        assert "tb2" in L.kernel_name
        L.upload(phi0)
        for _ in range(3):
            start = L.download()
            assert L.run_frame()
            assert not np.array_equal(L.download(), start)
        bad = L.download()
        bad[1, 2, 3] = np.float32(5e3)
        bad[-1, -1, -1] = np.float32("nan")
        L.upload(bad)
        assert not L.run_frame()
        back = L.download()
        ok = ~np.isnan(bad)
        assert np.array_equal(back[ok], bad[ok]) and np.isnan(back[-1, -1, -1])
        L.upload(_init(oracle_mod, shape, amp=0.2, seed=5))
        assert L.run_frame()


@pytest.mark.parametrize("path", ["mono", "rccl"])
def test_stable_frames_equal_raw_steps(gpu, oracle_mod, monkeypatch, path):
    """Frames that stay stable advance the field exactly as the same number of
    raw steps on the same noise counters: the frame instances of the kernels
    (guard flag, stability records, the snapshot store of the first fused
    launch) must not touch the trajectory (scripts/diag_frame_vs_steps.py)."""
    from stochquant_amd import unique_id
    shape = (256, 8, 16)
    phi0 = _init(oracle_mod, shape)

    def run(frames):
        kw = {}
        if path == "rccl":
            monkeypatch.setenv("SQ_GHOST", "4")
            kw = dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id())
        with _lat(shape, loops=6, **kw) as L:
            L.upload(phi0)
            if frames:
                for _ in range(3):
                    assert L.run_frame()
            else:
                L.step(18)
            return L.download()

    assert np.array_equal(run(True), run(False))


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("shape", [(256, 8, 16), (256, 16, 24)])
def test_frame_launches_equal_raw_steps_repeated(gpu, oracle_mod, monkeypatch, pipe, shape):
    """A frame of 4 steps equals 4 raw steps, repeated: the test that catches
    round 2's one-accumulator frame variant (a 16-byte store whose first data
    register a VALU overwrote at once: lanes 12-15 of every 16 of one output row
    stored the new value, in most runs; stochquant_amd/isa_check.py).  Both
    fused kernels (SQ_TB2_PIPE=1 pipelined, 0 round 2's)."""
    monkeypatch.setenv("SQ_TB2_PIPE", pipe)
    rng = np.random.default_rng(77)
    phi0 = (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)

    def run(frames):
        with _lat(shape, loops=4, dtau=0.02, m2=0.5, lam=1.0, seed=77) as L:
            L.upload(phi0)
            L.step(1)
            if frames:
                assert L.run_frame()
            else:
                L.step(4)
            return L.download()

    ref = run(False)
    for _ in range(8):
        assert np.array_equal(run(True), ref)


@pytest.mark.parametrize("shape,kw", [((256, 16, 24), {}), ((256, 64, 64), {}),
                                      ((256, 32, 40), {"comm": "loopback", "nslabs": 2})])
def test_neighbour_sync_equals_block_barrier(gpu, monkeypatch, shape, kw):
    """SQ_TB2_SYNC=p2p (row waves wait for their two neighbours' progress words
    instead of a block barrier per plane) gives the barrier kernel's field bit
    for bit, over repeated runs: a missing wait would read a neighbour's row of
    the wrong plane in some runs.  Plain and slab (ghost-zone) contexts."""
    monkeypatch.setenv("SQ_TB2_PIPE", "0")
    monkeypatch.setenv("SQ_FUSE2", "1")
    rng = np.random.default_rng(91)
    phi0 = (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)

    def run(sync, frame):
        monkeypatch.setenv("SQ_TB2_SYNC", sync)
        with _lat(shape, loops=8, dtau=0.01, m2=0.5, lam=1.0, seed=91, **kw) as L:
            L.upload(phi0)
            if frame:  # the frame kernels (records, fold) under either sync
                ok = L.run_frame()
                return L.download(), ok, L.dtau
            L.step(8)
            return L.download()

    ref = run("barrier", False)
    for _ in range(4):
        assert np.array_equal(run("p2p", False), ref)
    if not kw:
        fref = run("barrier", True)
        for _ in range(2):
            got = run("p2p", True)
            assert np.array_equal(got[0], fref[0]) and got[1:] == fref[1:]


RUN_FRAMES_CASES = [((256, 16, 16), 6, {}), ((256, 8, 12), 5, {}), ((64, 16, 8), 6, {}),
                    ((512, 8, 6), 4, {}), ((256, 8, 12), 6, {"comm": "loopback", "nslabs": 3})]


@pytest.mark.parametrize("tri", ["1", "0"])
@pytest.mark.parametrize("shape,loops,kw", RUN_FRAMES_CASES)
def test_run_frames_match_host_frames(gpu, oracle_mod, monkeypatch, shape, loops, kw, tri):
    """sq_run_frames (verdict, rollback and Δτ controller on the device between
    frames) and sq_run_frame per frame equal the host-decided
    frames (SQ_FRAME_HOST=1: record read-back, stab_rule and adapt on the host)
    bit for bit: verdicts, the Δτ after every frame, the field, the carried
    T / V and the last frame's records.  Δτ starts above the Euler limit, so
    the run mixes rolled-back frames (Δτ x 0.95) with stable ones (Δτ / 0.95
    after 11); fused (even and odd frame lengths), per-step, 512-wide and
    multi-slab (host path) contexts; three buffers (tri = 1, the default) and
    the snapshot fold path (SQ_FRAME_TRI=0: an unstable verdict rolls back by
    reading the padded snapshot and skips the snapshot store)."""
    nfr = 40
    monkeypatch.setenv("SQ_FRAME_TRI", tri)

    def run(mode):
        monkeypatch.setenv("SQ_FRAME_HOST", "1" if mode == "host" else "0")
        with _lat(shape, C=1.0, dtau=0.19, m2=1.0, lam=1.0, seed=99, loops=loops, **kw) as L:
            L.init_field(0.3)
            if mode == "batch":
                st, dt = L.run_frames(nfr)
            else:
                st, dt = [], []
                for _ in range(nfr):
                    st.append(L.run_frame())
                    dt.append(L.dtau)
                st, dt = np.array(st), np.array(dt)
            return st, dt, L.download(), L.stability(), L.step_counter

    ref = run("host")
    assert ref[0].any() and not ref[0].all(), ref[0]
    for mode in ("batch", "single"):
        got = run(mode)
        assert np.array_equal(got[0], ref[0]), mode
        assert np.array_equal(got[1], ref[1]), mode
        assert np.array_equal(got[2], ref[2]), mode
        for k in ("M", "D", "A"):
            assert np.array_equal(got[3][k], ref[3][k]), (mode, k)
        for k in ("fired", "T", "V"):
            assert got[3][k] == ref[3][k], (mode, k)
        assert got[4] == ref[4] == nfr * loops


def test_run_frames_after_upload_and_in_pieces(gpu, oracle_mod, monkeypatch):
    """A field uploaded by the caller (not yet through the guard) runs its first
    frame on the host path, the rest on the device; batches split anywhere
    (and a caller's Δτ / stability state set between them) give the frames of
    one batch."""
    shape, loops = (256, 8, 16), 4
    phi0 = _init(oracle_mod, shape, amp=0.3)

    def run(pieces):
        with _lat(shape, C=1.0, dtau=0.19, m2=1.0, lam=1.0, seed=5, loops=loops) as L:
            L.upload(phi0)
            st, dt = [], []
            for n in pieces:
                s, d = L.run_frames(n)
                st += list(s)
                dt += list(d)
            return np.array(st), np.array(dt), L.download(), L.dtau

    a = run([30])
    b = run([1, 7, 0, 13, 9])
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3] == b[3] == a[1][-1]
    monkeypatch.setenv("SQ_FRAME_HOST", "1")
    c = run([30])
    assert np.array_equal(a[0], c[0]) and np.array_equal(a[1], c[1]) and np.array_equal(a[2], c[2])


def test_block_stamps_are_two_steps(gpu, oracle_mod):
    """sq_phi4_block_stamps runs exactly the next two steps (one fused launch)
    and returns one start <= end stamp pair per block of that launch."""
    shape = (256, 16, 24)
    phi0 = _init(oracle_mod, shape, amp=0.3)
    with _lat(shape) as L, _lat(shape) as R:
        L.upload(phi0)
        R.upload(phi0)
        L.step(1)
        R.step(1)
        st, en = L.block_stamps()
        R.step(2)
        assert len(st) == len(en) > 0 and (en >= st).all() and (st > 0).all()
        # the same blocks' shader-clock counters: a clock between 100 MHz and 3 GHz
        cs, ce = L.block_clocks()
        assert len(cs) == len(st) and (ce >= cs).all()
        ok = en - st > 100  # blocks that ran >= 1 us of the 100 MHz clock
        assert ok.any()
        mhz = np.median((ce[ok] - cs[ok]) / (en[ok] - st[ok])) * 100.0
        assert 100.0 <= mhz <= 3000.0, mhz
        assert L.step_counter == R.step_counter == 3
        assert np.array_equal(L.download(), R.download())


HOT_256 = "phi4_tb2_kernel<true, false, 1, false, true, false>"


def test_c2_hot_instance_vs_oracle(gpu, oracle_mod, bm_tables):
    """The exact instance the bench times at 256^3 (VERDICT r4 next #1c), not
    a neighbour of it: a default context, the bench's init_field(0.1) (seed
    0x5EED, Δτ = 0.01, m² = λ = 1), 6 steps = 3 fused launches of
    phi4_tb2_kernel<true, false, 1, false, true, false> (the guard fast path on:
    the field came from init_field), compared with the oracle from the same
    initial field -- bitwise with the device's Box-Muller factors, within
    6 x the per-step bound (STEP_ATOL + STEP_RTOL |phi'|) of the mathematical
    normals.  The initial field itself is the oracle's phi4_init bit for bit
    in device-transcendental mode."""
    shape = (256, 256, 256)
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as L:
        L.init_field(0.1)
        phi0 = L.download()
        L.perf_reset()
        L.step(6)
        got = L.download()
        info = L.launch_info()
        perf = L.perf()
    assert info["kernel"] == HOT_256 and info["launches"] == 3, info
    assert info["grid"] == 512 * 640, info          # one round of 512 ten-wave blocks
    assert perf["fused_steps"] == 6 and perf["kernel_launches"] == 3
    p = oracle_mod.phi4_params(shape, 0.01, 1.0, 1.0, 0x5EED)
    with oracle_mod.device_transcendentals(bm_tables):
        assert np.array_equal(phi0, oracle_mod.phi4_init(p, 0.1))
        ref_dev = _oracle_run(oracle_mod, shape, phi0, 6, C=1.0, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
    assert np.array_equal(got, ref_dev), f"max diff {np.max(np.abs(got - ref_dev))}"
    del ref_dev
    ref = _oracle_run(oracle_mod, shape, phi0, 6, C=1.0, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
    err = np.abs(got.astype(np.float64) - ref)
    tol_report("c2_hot_instance", err, 6, ref, STEP_RTOL)
    assert np.all(err <= 6 * (STEP_ATOL + STEP_RTOL * np.abs(ref))), f"max err {err.max()}"


@pytest.mark.parametrize("shape,kw", [((256, 16, 40), {}), ((256, 16, 40), {"comm": "loopback", "nslabs": 3}),
                                      ((256, 16, 48), {"comm": "rccl"}), ((512, 8, 33), {}),
                                      ((64, 16, 24), {})])
def test_oracle_protocol_matches_oracle(gpu, oracle_mod, shape, kw):
    """bench.py's oracle_check protocol (verify.run_oracle_protocol: C = 0 set
    on the open context, the hash field uploaded, CHECK_STEPS steps) on small
    lattices, single slab / loopback slabs / RCCL self-exchange: the field is
    the oracle's bit for bit, and the context's noise comes back on."""
    from stochquant_amd import unique_id, verify
    if kw.get("comm") == "rccl":
        kw = dict(kw, nranks=1, rank=0, comm_id=unique_id())
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, **kw) as L:
        d = verify.run_oracle_protocol(L)
        got = L.download()
        assert L.params.C == 1.0
        L.init_field(0.1)
        L.step(2)
        noisy = L.download()
    p = oracle_mod.phi4_params(shape, 0.01, 1.0, 1.0, 0x5EED, C=0.0)
    ref = verify.hash_field(shape, 0, shape[2])
    for s in range(verify.CHECK_STEPS):
        ref = oracle_mod.phi4_step(p, ref, s)
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"
    assert d == verify.slab_digest(ref)
    if "comm_id" in kw:
        kw["comm_id"] = unique_id()
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, **kw) as L:   # the noise is back on
        L.init_field(0.1)
        L.step_counter = verify.CHECK_STEPS
        L.step(2)
        assert np.array_equal(L.download(), noisy)


@pytest.mark.parametrize("shape,kw", [((256, 16, 40), {}), ((256, 16, 40), {"comm": "loopback", "nslabs": 3}),
                                      ((256, 16, 48), {"comm": "rccl"}), ((64, 16, 24), {})])
def test_oracle_protocol_noise_matches_device_oracle(gpu, oracle_mod, bm_tables, shape, kw):
    """bench.py's oracle_check_noise protocol (C = 1, the hash field,
    CHECK_STEPS steps) on small lattices: the field is the oracle's in
    device-transcendental mode bit for bit, the digest is that field's, the
    context's C comes back, and the device tables hash as verify computes."""
    from stochquant_amd import unique_id, verify
    if kw.get("comm") == "rccl":
        kw = dict(kw, nranks=1, rank=0, comm_id=unique_id())
    with _lat(shape, C=0.5, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, **kw) as L:
        d = verify.run_oracle_protocol(L, noise=True)
        got = L.download()
        assert L.params.C == 0.5
    p = oracle_mod.phi4_params(shape, 0.01, 1.0, 1.0, 0x5EED, C=1.0)
    ref = verify.hash_field(shape, 0, shape[2])
    with oracle_mod.device_transcendentals(bm_tables):
        for s in range(verify.CHECK_STEPS):
            ref = oracle_mod.phi4_step(p, ref, s)
    assert np.array_equal(got, ref), f"max diff {np.max(np.abs(got - ref))}"
    assert d == verify.slab_digest(ref)
    assert verify.bm_tables_digest(verify.bm_tables(0)) == verify.bm_tables_digest(bm_tables)


def test_oracle_check_noise_full_size_256(gpu):
    """The bench's oracle_check_noise at N = 1 (256^3): the timed instance ran,
    the committed device-transcendental oracle digest matches; a flipped value
    fails."""
    from stochquant_amd import verify
    shape = (256, 256, 256)
    g = verify.load_oracle_golden()
    assert verify.NOISE_PREFIX + verify.golden_key(shape, 1) in g, "no committed noise digests"
    td = verify.bm_tables_digest(verify.bm_tables(0))
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as L:
        L.perf_reset()
        d = verify.run_oracle_protocol(L, noise=True)
        assert L.launch_info()["kernel"] == HOT_256
        bad = verify.run_oracle_protocol(L, corrupt=True, noise=True)
    assert verify.oracle_check_noise([d], [td], shape, 1) == "pass"
    assert verify.oracle_check_noise([bad], [td], shape, 1) == "fail"


def test_oracle_check_full_size_256(gpu):
    """The bench's oracle_check at N = 1 (256^3, the committed oracle digest of
    tests/golden/oracle_slabs.json): pass; a flipped value fails."""
    from stochquant_amd import verify
    shape = (256, 256, 256)
    with _lat(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as L:
        d = verify.run_oracle_protocol(L)
        bad = verify.run_oracle_protocol(L, corrupt=True)
    assert verify.oracle_check([d], shape, 1) == "pass"
    assert verify.oracle_check([bad], shape, 1) == "fail"


def test_launch_info_names_each_instance(gpu, monkeypatch):
    """sq_phi4_launch_info: the dominant step kernel's template instance and
    grid, per the launcher's own choice (the per-step kernel, the 512-wide
    pipelined fused kernel, the noise-off instance)."""
    with _lat((256, 16, 16), dtau=0.01) as L:
        L.step(4)
        assert L.launch_info()["kernel"].startswith("phi4_tb2_kernel<true, false, 1, false, true, false>")
        L.set_noise(0.0)
        L.perf_reset()
        L.step(4)
        assert L.launch_info()["kernel"] == "phi4_tb2_kernel<false, false, 1, false, true, false>"
        L.perf_reset()
        assert L.launch_info() == {"kernel": "", "grid": 0, "launches": 0}
    with _lat((512, 8, 16), dtau=0.01) as L:
        L.step(2)
        assert L.launch_info()["kernel"] == "phi4_tb2p_kernel<true, true, 6, false, true>"
    monkeypatch.setenv("SQ_FUSE2", "0")
    with _lat((32, 32, 32), dtau=0.01) as L:
        L.step(3)
        info = L.launch_info()
        # 32-site rows: 8 lanes x 4 sites per row (QX = 8), one row per lane, packed-free scalar arithmetic
        assert info["kernel"] == "phi4_step_kernel<8, 1, 1, false, true, 1, false>" and info["launches"] == 3, info
        assert L.kernel_name.startswith(info["kernel"][:-len(", false>")] + ">"), (L.kernel_name, info)


@pytest.mark.parametrize("shape,kw", [((256, 16, 24), {}), ((32, 8, 13), {}), ((256, 8, 30), {"comm": "loopback", "nslabs": 4}),
                                      ((64, 16, 12), {"comm": "rccl"})])
def test_init_field_hash_matches_host(gpu, shape, kw):
    """sq_init_field_hash on the device is verify.hash_field (numpy) bit for
    bit, slab by slab: the oracle's digests start from the same field."""
    from stochquant_amd import unique_id, verify
    if kw.get("comm") == "rccl":
        kw = dict(kw, nranks=1, rank=0, comm_id=unique_id())
    with _lat(shape, **kw) as L:
        L.init_field_hash(verify.HASH_FIELD_AMP, verify.HASH_FIELD_KEY)
        got = L.download()
        L.init_field_hash(0.5, 12345)
        other = L.download()
    assert np.array_equal(got, verify.hash_field(shape, 0, shape[2]))
    assert not np.array_equal(other, got) and np.abs(other).max() <= 0.5
