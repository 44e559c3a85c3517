"""Kernel trace of short timed regions (the driver's --steps 20): five
step(200) / sync / step(20) / sync rounds, for rocprofv3 --kernel-trace; the
gaps between the K = 20 region's kernels come from the trace.
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 scripts/diag_k20_trace.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stochquant_amd import Phi4Lattice
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as lat:
        lat.init_field(0.1)
        lat.step(2000)
        lat.sync()
        for _ in range(5):
            lat.step(200)
            torch.cuda.synchronize()
            lat.step(20)
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
