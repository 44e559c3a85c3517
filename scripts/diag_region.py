"""Where the driver's K = 20 timed region loses time against the kernel stream
(17.43 us/step wall vs 15.51 on the kernel stream).

Interleaved repetitions on one 256^3 lattice after a clock settle; medians of:
  wall_K      sync; t0; step(K); torch.cuda.synchronize(); t1     (bench's region)
  wall_K_lib  the same, ending with the library's stream sync
  host_K      time for step(K) to return (host launch cost)
  empty       sync; t0; torch.cuda.synchronize(); t1
  ev_K        one hipEvent pair around step(K) on the kernel stream (mode 2)
for K in {2, 20, 200}.

    python scripts/diag_region.py [--reps 40]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--flags", default="none", choices=["none", "auto", "spin", "yield", "block"],
                    help="hipSetDeviceFlags schedule before the device is first used")
    a = ap.parse_args()
    if a.flags != "none":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        fl = {"auto": 0, "spin": 1, "yield": 2, "block": 4}[a.flags]
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(fl))
        print(json.dumps({"hipSetDeviceFlags": a.flags, "rc": rc}), flush=True)
    import torch
    from stochquant_amd import Phi4Lattice, _lib
    torch.cuda.set_device(0)
    L = a.size
    lat = Phi4Lattice((L, L, L), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, device=0)
    lat.init_field(0.1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.5:
        lat.step(50)
        lat.sync()
    res = {}

    def rec(k, v):
        res.setdefault(k, []).append(v)

    for _ in range(a.reps):
        for K in (2, 20, 200):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lat.step(K)
            th = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rec(f"wall_{K}", (t1 - t0) * 1e6)
            rec(f"host_{K}", (th - t0) * 1e6)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lat.step(K)
            lat.sync()
            t1 = time.perf_counter()
            rec(f"wall_{K}_lib", (t1 - t0) * 1e6)
            lat.perf_reset()
            lat.set_profiling(2)
            torch.cuda.synchronize()
            lat.step(K)
            torch.cuda.synchronize()
            lat.sync()
            p = lat.perf()
            lat.set_profiling(0)
            rec(f"ev_{K}", p["step_kernel_ms"] * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rec("empty", (t1 - t0) * 1e6)
        t0 = time.perf_counter()
        lat.step(0)
        rec("host_0", (time.perf_counter() - t0) * 1e6)
        t0 = time.perf_counter()
        _lib.load().sq_abi_version()
        rec("host_abi", (time.perf_counter() - t0) * 1e6)
    out = {"flags": a.flags}
    out.update({k: round(statistics.median(v), 2) for k, v in res.items()})
    for K in (2, 20, 200):
        out[f"overhead_{K}_us"] = round(out[f"wall_{K}"] - out[f"ev_{K}"], 2)
        out[f"wall_per_step_{K}"] = round(out[f"wall_{K}"] / K, 3)
    print(json.dumps(out), flush=True)
    lat.close()


if __name__ == "__main__":
    main()
