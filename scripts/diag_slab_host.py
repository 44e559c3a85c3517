"""Is the slab path host-bound?  For the single lattice and the one-GPU slab
transports (RCCL / P2P self-exchange, G = 16), after a clock settle, medians of
  host_K   time for step(K) to return (the host's issue cost: launches, event
           records and waits, the RCCL calls)
  wall_K   step(K) + device synchronise
per step, for K in {16, 320, 2000}.  If host_K / K approaches wall_K / K the
GPU waits for the host, and a graph of the 16-step block is the lever.

    python scripts/diag_slab_host.py [--reps 5]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--comms", default="none,rccl,p2p")
    a = ap.parse_args()
    import torch
    from stochquant_amd import Phi4Lattice, unique_id
    torch.cuda.set_device(0)
    L = a.size
    for comm in a.comms.split(","):
        kw = dict(dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, device=0)
        if comm == "rccl":
            lat = Phi4Lattice((L, L, L), comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
        elif comm == "p2p":
            lat = Phi4Lattice((L, L, L), comm="p2p", nranks=1, rank=0, **kw)
            lat.p2p_connect([lat.p2p_handle()])
        else:
            lat = Phi4Lattice((L, L, L), **kw)
        lat.init_field(0.1)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.5:
            lat.step(64)
            lat.sync()
        res = {}
        for _ in range(a.reps):
            for K in (16, 320, 2000):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lat.step(K)
                th = time.perf_counter()
                lat.sync()
                t1 = time.perf_counter()
                res.setdefault(f"host_{K}", []).append((th - t0) * 1e6 / K)
                res.setdefault(f"wall_{K}", []).append((t1 - t0) * 1e6 / K)
        out = {"comm": comm, "ghost": getattr(lat, "ghost", None), "unit": "us per step"}
        out.update({k: round(statistics.median(v), 3) for k, v in sorted(res.items())})
        print(json.dumps(out), flush=True)
        lat.close()


if __name__ == "__main__":
    main()
