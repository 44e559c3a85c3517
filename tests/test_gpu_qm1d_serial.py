"""SQ_ORDER_SERIAL: the reference's own serial semantics on the MI355X
 against the serial oracle (oracle/orc_qm1d.c
orc_serial_launch, pinned bit-exact to the reference's recorded outputs).

  * LCG stream: the integer words, seeds and xi of the reference's random()
    (tau_kernel.cl:269-284) are bit-identical: the device evaluates glibc's
    own logf / cosf algorithms (csrc/sq_glibcf.h, tests/test_glibcf.py), not
    correctly rounded ones (glibc's differ from correct rounding by 1 ulp in
    ~1 % of arguments).
  * Every frame (stable or broken), with injected or device-drawn noise, is
    bit-identical: field, running means, omega, lrgEl, lrgVl, Δτ, the calls
    consumed -- potID 3's x_cl = eta tanhf(...) included (glibc's tanhf,
    restated the same way; the hardware's differs by 1 ulp in ~14 % of
    arguments).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gpu_lcg(sqlib, seed, N, loops, generator=1):
    import ctypes
    n = (N + 1) * loops
    w1 = np.empty(n, dtype=np.uint32)
    w2 = np.empty(n, dtype=np.uint32)
    seeds = np.empty(n, dtype=np.uint64)
    xi = np.empty(n)
    P = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))
    rc = sqlib.sq_selftest_lcg(0, seed, N, loops, P(w1, ctypes.c_uint), P(w2, ctypes.c_uint),
                               P(seeds, ctypes.c_ulonglong), P(xi, ctypes.c_double), generator)
    assert rc == 0
    return xi, w1, w2, seeds


@pytest.mark.parametrize("generator", [0, 1])
@pytest.mark.parametrize("seed,N,loops", [(12345, 4, 2), (1804289383, 100, 30), (7, 3, 500),
                                          (2 ** 31 - 3, 1000, 4), (1804289383, 999, 1000)])
def test_lcg_stream_matches_reference(gpu, sqlib, oracle_mod, seed, N, loops, generator):
    xi, w1, w2, seeds = _gpu_lcg(sqlib, seed, N, loops, generator)
    rxi, rw1, rw2, rseeds = oracle_mod.ref_noise_stream(seed, N, loops)
    assert np.array_equal(w1, rw1) and np.array_equal(w2, rw2) and np.array_equal(seeds, rseeds)
    assert np.array_equal(xi, rxi)


def _run_pair(oracle_mod, N, a, dtau, pot, C, loops, seed, frames, f0, inject=True, omega=None,
              check=None):
    from stochquant_amd import Qm1dChain
    omega = a * (N // 2) if omega is None else omega
    ch = oracle_mod.SerialChain(N, a, dtau, pot, C, loops, seed, f0, omega=omega)
    results = []
    with Qm1dChain(N, a, dtau, pot=pot, C=C, loops=loops, ordering="serial", lcg_seed=seed) as g:
        g.upload(f0, omega=omega)
        for fr in range(frames):
            xi, _, _, seeds = oracle_mod.ref_noise_stream(ch.d.seed, N, loops)
            if inject:
                g.inject_noise(xi)
            s_o = ch.frame()
            s_g = g.run_frame()
            d = g.download()
            sc = g.scan
            res = dict(frame=fr, stable=(s_o, int(s_g)), dtau=(ch.d.dtau, g.dtau),
                       lrgEl=(ch.d.lrgEl, sc["lrgEl"]), lrgVl=(ch.d.lrgVl, sc["lrgVl"]),
                       omega=(ch.omega, d["omega"]), runs=(ch.runs, d["runs"]),
                       seed=(ch.d.seed, int(seeds[g.noise_consumed - 1])),
                       f=(ch.host["f"].copy(), d["f"]), x=(ch.host["x"].copy(), d["x"]),
                       xx0=(ch.host["xx0"].copy(), d["xx0"]))
            if not inject:
                res["seed"] = (ch.d.seed, g.lcg_seed)
            results.append(res)
            if check:
                check(res)
    return results


def _exact(res):
    for k in ("stable", "dtau", "lrgEl", "lrgVl", "omega", "runs", "seed"):
        assert res[k][0] == res[k][1], (res["frame"], k, res[k])
    for k in ("f", "x", "xx0"):
        assert np.array_equal(res[k][0], res[k][1]), (res["frame"], k, np.max(np.abs(res[k][0] - res[k][1])))


@pytest.mark.parametrize("N,loops,dtau", [(2, 3, 0.01), (3, 1, 0.01), (4, 2, 0.01), (5, 7, 0.02),
                                          (63, 20, 0.01), (64, 20, 0.01), (65, 9, 0.01), (100, 50, 0.002),
                                          (129, 13, 0.01), (200, 40, 0.004), (1000, 8, 0.001),
                                          (3072, 3, 0.001), (4096, 2, 0.001)])
def test_injected_noise_frames_bitwise_pot0(gpu, oracle_mod, N, loops, dtau):
    rng = np.random.default_rng(N)
    f0 = 0.3 * rng.standard_normal(N)
    res = _run_pair(oracle_mod, N, 0.1, dtau, 0, 1.0, loops, 1804289383 + N, 6, f0, check=_exact)
    assert any(r["stable"][0] == 1 for r in res)


def test_injected_noise_unstable_frames_bitwise(gpu, oracle_mod):
    """dtau/dt^2 = 5 (the reference presets' regime): frames break mid-way,
    dtau shrinks, the seed advances by the calls made before the break."""
    N, a = 40, 0.1
    f0 = np.random.default_rng(3).standard_normal(N)
    res = _run_pair(oracle_mod, N, a, 5 * a * a, 0, 1.0, 25, 42, 70, f0, check=_exact)
    assert any(r["stable"][0] == 0 for r in res) and any(r["stable"][0] == 1 for r in res)


def test_appendix_c_shape_bitwise(gpu, oracle_mod):
    """The survey's recorded run (N=4, a=0.5, dtau=0.01, loops=5) frame by frame."""
    rng = np.random.default_rng(0)
    res = _run_pair(oracle_mod, 4, 0.5, 0.01, 0, 1.0, 5, 1714636915, 10, 0.1 * rng.standard_normal(4),
                    check=_exact)
    assert len(res) == 10


@pytest.mark.parametrize("N,loops,dtau,frames", [(100, 40, 0.002, 5), (40, 25, 0.05, 40), (1000, 8, 0.001, 3)])
def test_device_draws_frames_bitwise(gpu, oracle_mod, N, loops, dtau, frames):
    """GPU-generated draws (the product's default): every frame bitwise,
    unstable ones (dtau/dt^2 = 5) included."""
    f0 = 0.2 * np.random.default_rng(N).standard_normal(N)
    res = _run_pair(oracle_mod, N, 0.1, dtau, 0, 1.0, loops, 987654321 + N, frames, f0, inject=False,
                    check=_exact)
    assert len(res) == frames


@pytest.mark.parametrize("inject", [True, False])
def test_double_well_bitwise(gpu, oracle_mod, inject):
    """potID 3 (x_cl = eta tanhf(...), glibc's tanhf on the device)."""
    N, loops = 64, 20
    f0 = 0.1 * np.random.default_rng(9).standard_normal(N)
    _run_pair(oracle_mod, N, 0.1, 0.001, 3, 1.0, loops, 31337, 4, f0, inject=inject, check=_exact)


def test_serial_order_rejects_large_n(gpu):
    from stochquant_amd import Qm1dChain, StochQuantError
    with Qm1dChain(4097, 0.1, 0.001, pot=0, loops=2) as g:
        with pytest.raises(StochQuantError):
            g.set_ordering("serial")


@pytest.mark.parametrize("generator", [0, 1])
def test_lcg_exceptional_calls(gpu, sqlib, oracle_mod, generator):
    """Seeds that drive the rare branches of random(): case P (s < 2^31 and
    t2 < 2^31 -> s + t2) and the u64 wrap of t2 - 2^31.  The parallel-prefix
    generator's exact fix-up must reproduce the serial chain bit for bit."""
    M = (1 << 48) - 1
    A, B = 0x5DEECE66D, 0xB
    found = []
    # search small seeds whose first call has t2 < 2^31 (case P from a small seed)
    for s in range(1, 3_000_000):
        t1 = ((s + 0) * A + B) & M
        t2 = ((t1 + 0) * A + B) & M
        if t2 < 2 ** 31:
            found.append(s)
            if len(found) == 2:
                break
    assert found
    for seed in found:
        xi, w1, w2, seeds = _gpu_lcg(sqlib, seed, 7, 300, generator)
        rxi, rw1, rw2, rseeds = oracle_mod.ref_noise_stream(seed, 7, 300)
        assert np.array_equal(w1, rw1) and np.array_equal(w2, rw2) and np.array_equal(seeds, rseeds)
        assert np.array_equal(xi, rxi)


_M48 = (1 << 48) - 1
_A, _B = 0x5DEECE66D, 0xB


def _seed_reaching(s_k, k, N):
    """The seed whose case-Q chain (s' = A^2 s + beta(g), the common branch of
    tau_kernel.cl:269-284) is s_k before call k: the chain run backwards."""
    alpha = _A * _A & _M48
    ainv = pow(alpha, -1, 1 << 48)
    s = s_k
    for j in range(k - 1, -1, -1):
        g = j % (N + 1)
        beta = (_A * _A * g + _A * _B + _A * g + _B - 2 ** 31) & _M48
        s = ainv * (s - beta) & _M48
    return s


@pytest.mark.parametrize("kind,k", [("retry", 500_123), ("retry", 16_000), ("retry", 999_999),
                                    ("case_p", 333_333), ("case_p", 61)])
def test_lcg_exception_mid_stream(gpu, sqlib, oracle_mod, kind, k):
    """An exceptional call deep inside a 10^6-call launch (constructed by
    running the chain backwards from a state that takes it): the isinf retry
    (t1 >> 16 == 0) or case P (s < 2^31 and t2 < 2^31).  The grid-wide
    generator's chunks after it are invalid; the one-block resume from the
    first exceptional call must give the serial chain bit for bit."""
    N, loops = 999, 1000
    g = k % (N + 1)
    if kind == "retry":
        s_k = ((12345 - _B) * pow(_A, -1, 1 << 48) - g) & _M48  # t1 = 12345 -> t1 >> 16 == 0
    else:
        s_k = next(s for s in range(1, 1 << 31)
                   if ((((s + g) * _A + _B) & _M48) + g) * _A + _B & _M48 < 2 ** 31)
    seed = _seed_reaching(s_k, k, N)
    rxi, rw1, rw2, rseeds = oracle_mod.ref_noise_stream(seed, N, loops)
    assert int(rseeds[k - 1]) & _M48 == s_k  # the construction reached the state
    for generator in (1, 0):
        xi, w1, w2, seeds = _gpu_lcg(sqlib, seed, N, loops, generator)
        assert np.array_equal(w1, rw1) and np.array_equal(w2, rw2) and np.array_equal(seeds, rseeds)
        assert np.array_equal(xi, rxi)
