"""Per-block start / end stamps of the last fused launch (diagnostic build
with g_tb_stamp, s_memrealtime at 100 MHz): how much of a launch is ramp,
tail and block imbalance.   SQ_LIB=<diag .so> python scripts/diag_tb_stamps.py [L]

The diagnostic build (scripts/build_variant.py on a patched sq_phi4.hip) adds
    __device__ unsigned long long g_tb_stamp[2 * 65536];
a store of __builtin_amdgcn_s_memrealtime() into g_tb_stamp[2b] by thread 0
of block b at the top of phi4_tb2_kernel and into g_tb_stamp[2b+1] after a
__syncthreads() at its end, and
    extern "C" int sq_diag_tb_stamps(unsigned long long *out, int n)
copying the symbol out (hipMemcpyFromSymbol).  Results: profiles/r02/block_stamps/."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    from stochquant_amd import Phi4Lattice, _lib
    lib = _lib.load()
    with Phi4Lattice((L, L, L), dtau=0.01, m2=1.0, lam=1.0) as lat:
        lat.init_field(0.1)
        lat.step(2000 if L <= 256 else 200)
        lat.sync()
        for rep in range(3):
            lat.step(2)
            lat.sync()
            nb = 512
            a = np.zeros(2 * nb, dtype=np.uint64)
            assert lib.sq_diag_tb_stamps(a.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), nb) == 0
            st, en = a[0::2].astype(np.int64), a[1::2].astype(np.int64)
            t0 = st.min()
            s, e = (st - t0) * 10e-3, (en - t0) * 10e-3   # us
            d = e - s
            print(f"L={L} rep {rep}: launch span {e.max():.2f} us; starts {s.min():.2f}..{s.max():.2f} "
                  f"(p50 {np.median(s):.2f}); ends {e.min():.2f}..{e.max():.2f} (p10 {np.percentile(e, 10):.2f}, "
                  f"p50 {np.median(e):.2f}, p90 {np.percentile(e, 90):.2f}); block duration mean {d.mean():.2f} "
                  f"min {d.min():.2f} max {d.max():.2f}; busy fraction {d.sum() / (nb * e.max()):.3f}", flush=True)


if __name__ == "__main__":
    main()
