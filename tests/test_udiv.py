"""The QM1D kernels' shared-divisor division (sq_qm1d.hip udiv) is the
compiler's fp64 division expansion with the divisor's refined reciprocal
computed once; this CPU check runs that arithmetic (C fma is exact) with the
initial reciprocal up to 4 ulp off, as v_rcp_f64's approximation may be, over
udiv's fast range, and requires every quotient to equal IEEE a / b.  The GPU
side is pinned by the bitwise QM1D frame tests (test_gpu_qm1d.py)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_udiv_correctly_rounded(tmp_path):
    exe = str(tmp_path / "udiv_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "udiv_check.c"), "-lm"],
                   check=True)
    r = subprocess.run([exe, "3000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "bad 0" in r.stdout
