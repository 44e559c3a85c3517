"""Diagnostics for the phi^4 step kernel on one GPU.

    python scripts/diag_phi4.py copy               # copy ceiling vs working-set size
    python scripts/diag_phi4.py steps [--size 256] [--steps 50] [--C 1]
        (run under rocprofv3 --pmc ... to collect counters for the step kernel)
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["copy", "steps"])
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--C", type=float, default=1.0)
    ap.add_argument("--sizes", default="", help="copy: buffer sizes in MiB (comma list)")
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice, _lib
    lib = _lib.load()
    if a.what == "copy":
        sizes = [int(v) for v in a.sizes.split(",")] if a.sizes else [16, 32, 64, 96, 128, 256, 512, 1024, 2048]
        for mib in sizes:
            g = ctypes.c_double()
            iters = max(10, int(20 * 1024 / mib))
            rc = lib.sq_copy_bandwidth(0, mib << 20, iters, ctypes.byref(g))
            print(json.dumps({"buffer_MiB": mib, "working_set_MiB": 2 * mib, "copy_GBps": round(g.value, 1),
                              "rc": rc}), flush=True)
        return
    L = a.size
    lat = Phi4Lattice((L, L, L), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, C=a.C)
    lat.init_field(0.1)
    lat.step(a.steps)
    lat.sync()
    print(json.dumps({"size": L, "steps": a.steps, "tile": lat.tile}))
    lat.close()


if __name__ == "__main__":
    main()
