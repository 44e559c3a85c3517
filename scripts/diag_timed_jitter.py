"""Spread of the driver's 20-step timed region under host-side settings:
default, Python's garbage collector off, and the process pinned to one CPU
(with the collector off).  40 regions each, interleaved.
    python scripts/diag_timed_jitter.py"""
import gc
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stochquant_amd import Phi4Lattice
    cpus0 = os.sched_getaffinity(0)
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as lat:
        lat.init_field(0.1)
        lat.step(4000)
        lat.sync()
        res = {"default": [], "gc_off": [], "pinned_gc_off": []}
        for _ in range(40):
            for mode in res:
                if mode != "default":
                    gc.disable()
                if mode == "pinned_gc_off":
                    os.sched_setaffinity(0, {min(cpus0)})
                lat.step(200)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lat.step(20)
                torch.cuda.synchronize()
                res[mode].append((time.perf_counter() - t0) * 1e6)
                os.sched_setaffinity(0, cpus0)
                gc.enable()
        for mode, v in res.items():
            v = np.array(v)
            print(f"{mode:14s} min {v.min():7.1f}  p10 {np.percentile(v, 10):7.1f}  median {np.median(v):7.1f}  "
                  f"p90 {np.percentile(v, 90):7.1f}  max {v.max():7.1f} us", flush=True)


if __name__ == "__main__":
    main()
