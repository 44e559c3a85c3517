"""Wall time of K = 20 steps at 256^3 under different host-side completion
waits (torch.cuda.synchronize = hipDeviceSynchronize, the library's stream
synchronise, both), alternating, after a clock-settle phase."""
import statistics
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from stochquant_amd import Phi4Lattice  # noqa: E402

torch.cuda.set_device(0)
lat = Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
lat.init_field(0.1)
t = time.perf_counter()
while time.perf_counter() - t < 1.5:
    lat.step(50)
    lat.sync()
res = {"torch": [], "lib": [], "lib+torch": []}
for rep in range(30):
    for mode in res:
        lat.step(10)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lat.step(20)
        if mode in ("lib", "lib+torch"):
            lat.sync()
        if mode in ("torch", "lib+torch"):
            torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e6 / 20)
for mode, v in res.items():
    print(f"{mode:10s} median {statistics.median(v):.2f} us/step  min {min(v):.2f}")
