"""Device building blocks: Philox bits (KAT, bit-exact), DPP lane rotation,
Box-Muller normals vs the oracle's double-evaluated values."""
import ctypes

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

# |xi_gpu - xi_oracle| bound for the hardware-transcendental Box-Muller
# (v_log_f32 / v_sqrt_f32 / v_sin_f32 / v_cos_f32, each ~1 ulp) against the
# double-evaluated, once-rounded value: absolute 2e-6 + relative 2e-6.
NORMAL_ATOL = 2e-6
NORMAL_RTOL = 2e-6


def test_philox_kat_on_device(gpu, sqlib):
    for v in golden("philox_kat.json")["vectors"]:
        ctr = (ctypes.c_uint * 4)(*[int(x, 16) for x in v["ctr"]])
        key = (ctypes.c_uint * 2)(*[int(x, 16) for x in v["key"]])
        out = (ctypes.c_uint * 4)()
        assert sqlib.sq_selftest_philox(0, ctr, key, out) == 0
        assert [f"{o:08x}" for o in out] == v["out"]


def test_dpp_wave_rotation(gpu, sqlib):
    out = (ctypes.c_float * 128)()
    assert sqlib.sq_selftest_dpp(0, out) == 0
    a = np.array(out[:])
    lanes = np.arange(64)
    assert np.array_equal(a[:64], (lanes - 1) % 64)   # wave_ror:1  lane i <- i-1
    assert np.array_equal(a[64:], (lanes + 1) % 64)   # wave_rol:1  lane i <- i+1


@pytest.mark.parametrize("stream,quad0,step", [(0, 0, 0), (0, 123456789, 77), (1, 0, 5), (2, 2**40 + 3, 2**33 + 9)])
def test_normals_match_oracle(gpu, sqlib, oracle_mod, stream, quad0, step):
    n = 4096
    seed = 0x1234_5678_9ABC
    out = np.empty(4 * n, np.float32)
    rc = sqlib.sq_selftest_normals(0, seed, stream, quad0, step,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n)
    assert rc == 0
    ref = oracle_mod.normals(seed, stream, quad0, step, n)
    err = np.abs(out.astype(np.float64) - ref)
    bound = NORMAL_ATOL + NORMAL_RTOL * np.abs(ref)
    print("max normal err", err.max(), "max rel", (err / (np.abs(ref) + 1e-30)).max())
    assert np.all(err <= bound)


def test_bm_tables_accuracy(gpu, bm_tables):
    """The device's Box-Muller factors (the tables the oracle's
    device-transcendental mode uses) against the double-evaluated functions:
    v_log_f32 / v_sqrt_f32 / v_cos_f32 / v_sin_f32 of every 23-bit argument."""
    n = 1 << 23
    m = np.arange(n, dtype=np.float64)
    u = 1.0 - m * 2.0 ** -23
    t = m * 2.0 ** -23
    rad, radq, cs, sn = (bm_tables[k * n:(k + 1) * n].astype(np.float64) for k in range(4))
    r_ex = np.sqrt(-2.0 * np.log(u))
    rq_ex = np.sqrt(-np.log2(u))
    for got, ex in ((rad, r_ex), (radq, rq_ex)):
        assert np.all(np.abs(got - ex) <= 1e-6 + 1e-6 * ex)
    assert np.all(np.abs(cs - np.cos(2 * np.pi * t)) <= 2e-6)
    assert np.all(np.abs(sn - np.sin(2 * np.pi * t)) <= 2e-6)
    print("max |r - exact| rel", np.max(np.abs(rad - r_ex) / np.maximum(r_ex, 1e-30)),
          "max |cos - exact|", np.max(np.abs(cs - np.cos(2 * np.pi * t))))


def test_copy_bandwidth_runs(gpu, sqlib):
    g = ctypes.c_double()
    assert sqlib.sq_copy_bandwidth(0, 1 << 28, 10, ctypes.byref(g)) == 0
    print("copy GB/s", g.value)
    assert g.value > 1000
