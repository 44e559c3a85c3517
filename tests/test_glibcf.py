"""The serial order's float transcendentals (csrc/sq_glibcf.h: glibc 2.35's
logf / cosf / tanhf algorithms restated for the device) against this host's
libm -- the libm the reference's random() and clas() run on
(tau_kernel.cl:222,276-277) and the oracle calls.  CPU: the header compiled
for the host by scripts/glibc_f32_check.c over every 3rd float of the ranges
(the script's default stride 1 is the exhaustive run, 0 mismatches, DESIGN.md
§4.1).  GPU: the device build on strided samples, bit for bit."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_restatement_matches_host_libm(tmp_path):
    exe = tmp_path / "glibc_f32_check"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "scripts", "glibc_f32_check.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "3"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count(" 0 of ") == 3


def _args(fn):
    u = np.arange(0, 2 ** 32, 61, dtype=np.uint64)
    x = u.astype(np.uint32).view(np.float32)
    if fn == 0:    # logf: [0, 2) and the specials
        x = np.concatenate([x[(x >= 0) & (x < 2)], np.array([0.0, -0.0, 1.0, np.inf], np.float32)])
    elif fn == 1:  # cosf: |x| <= 6.3 (2 * 3.1415 * u)
        x = x[np.abs(x) <= 6.3]
    else:          # tanhf: every 61st float, NaNs aside
        x = x[~np.isnan(x)]
    return np.ascontiguousarray(x)


@pytest.mark.gpu
@pytest.mark.parametrize("fn", [0, 1, 2], ids=["logf", "cosf", "tanhf"])
def test_device_matches_host_libm(gpu, sqlib, oracle_mod, fn):
    x = _args(fn)
    y = np.empty_like(x)
    F = ctypes.POINTER(ctypes.c_float)
    assert sqlib.sq_selftest_libm(0, fn, x.ctypes.data_as(F), y.ctypes.data_as(F), x.size) == 0
    ref = oracle_mod.libm_f32(fn, x)
    same = y.view(np.uint32) == ref.view(np.uint32)
    print(x.size, "arguments,", int((~same).sum()), "differ")
    assert same.all(), x[~same][:8]
