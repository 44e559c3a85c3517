"""Where the fixed cost of a short timed region goes (the driver's --steps 20):
wall time of K fused steps bracketed by torch.cuda.synchronize() against the
kernels' own span, for K = 20 and 2000, and the pieces: the host's enqueue
call, an idle synchronize, a one-launch round trip.
    python scripts/diag_timed_overhead.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stochquant_amd import Phi4Lattice
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as lat:
        lat.init_field(0.1)
        lat.step(4000)
        lat.sync()
        torch.cuda.synchronize()
        res = {}
        for K in (2, 20, 200, 2000):
            ws, enq = [], []
            for _ in range(15):
                lat.step(200)          # busy chip, as in the bench's settle
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lat.step(K)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                ws.append((t2 - t0) * 1e6)
                enq.append((t1 - t0) * 1e6)
            res[K] = (np.median(ws), np.min(ws), np.median(enq))
            print(f"K={K:5d}: wall median {res[K][0]:9.1f} us  min {res[K][1]:9.1f}  per step {res[K][0] / K:7.3f}  "
                  f"enqueue call {res[K][2]:7.1f} us", flush=True)
        per = (res[2000][0] - res[200][0]) / 1800
        print(f"marginal per step (2000 vs 200): {per:.3f} us; fixed cost at K=20: {res[20][0] - 20 * per:.1f} us")
        idle = []
        for _ in range(20):
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            idle.append((time.perf_counter() - t0) * 1e6)
        print(f"idle torch.cuda.synchronize: median {np.median(idle):.1f} us")
        idle = []
        for _ in range(20):
            t0 = time.perf_counter()
            lat.sync()
            idle.append((time.perf_counter() - t0) * 1e6)
        print(f"idle lat.sync: median {np.median(idle):.1f} us")


if __name__ == "__main__":
    main()
