"""Per-plane max |difference| between the single-slab run (one step per
launch) and a slab run with fused inner steps -- a debugging aid.

    python scripts/diag_fuse_slab.py [--comm rccl|loopback] [--ghost 4] [--steps 4] [--shape 256,8,16]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comm", default="rccl")
    ap.add_argument("--ghost", default="4")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--shape", default="256,8,16")
    ap.add_argument("--nslabs", type=int, default=2)
    ap.add_argument("--C", type=float, default=1.0)
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice, unique_id
    shape = tuple(int(v) for v in a.shape.split(","))
    rng = np.random.default_rng(5)
    phi0 = (0.5 * rng.standard_normal(shape[::-1])).astype(np.float32)
    kw = dict(dtau=0.02, m2=0.5, lam=1.0, seed=1234, C=a.C)
    os.environ["SQ_FUSE2"] = "0"
    with Phi4Lattice(shape, **kw) as L:
        L.upload(phi0)
        L.step(a.steps)
        mono = L.download()
    os.environ["SQ_FUSE2"] = "1"
    os.environ["SQ_GHOST"] = a.ghost
    extra = dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id()) if a.comm == "rccl" else \
        dict(comm="loopback", nslabs=a.nslabs)
    with Phi4Lattice(shape, **kw, **extra) as L:
        print(L.kernel_name, L.ghost)
        L.upload(phi0)
        L.step(a.steps)
        got = L.download()
    d = np.abs(got.astype(np.float64) - mono).max(axis=(1, 2))
    print("per-plane max diff:", " ".join(f"{z}:{v:.2e}" for z, v in enumerate(d) if v > 0) or "none")


if __name__ == "__main__":
    main()
