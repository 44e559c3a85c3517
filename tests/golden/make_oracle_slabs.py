"""Oracle digests for bench.py's `oracle_check` (stochquant_amd/verify.py) --
test infrastructure: runs the CPU oracle (oracle/orc_phi4.c, the reference's
per-site update tau_kernel.cl:111-117 restated for the 3-D φ⁴ lattice) with
the noise off on the bench's lattices and writes, per rank count N, the
blake2b digest of every rank's slab after verify.CHECK_STEPS steps from
verify.hash_field.  No GPU is involved: these are the oracle's bits, which
the GPU must reproduce exactly (C = 0 is deterministic fp32 arithmetic).

Lattices: the weak-scaling 256 x 256 x 256N (N = 1, 2, 4, 8; every rank a
256^3 slab) and the strong-scaling 1024^3 (N = 1, 2, 4, 8).

    python tests/golden/make_oracle_slabs.py [--threads T] [--quick]

(--quick: the weak lattices only.)  Output: tests/golden/oracle_slabs.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (test infrastructure)
from stochquant_amd import verify  # noqa: E402
from stochquant_amd.decomp import slab_bounds  # noqa: E402


def oracle_run(shape, threads):
    P = verify.CHECK_PARAMS
    p = oracle.phi4_params(shape, P["dtau"], P["m2"], P["lam"], P["seed"], C=0.0)
    phi = verify.hash_field(shape, 0, shape[2])
    for s in range(verify.CHECK_STEPS):
        phi = oracle.phi4_step(p, phi, s, threads)
    return phi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    oracle.build()
    out = verify.load_oracle_golden()
    cases = [((256, 256, 256 * n), [n]) for n in (1, 2, 4, 8)]
    if not a.quick:
        cases.append(((1024, 1024, 1024), [1, 2, 4, 8]))
    P = verify.CHECK_PARAMS
    for shape, ns in cases:
        t0 = time.time()
        f = oracle_run(shape, a.threads)
        for n in ns:
            slabs = [verify.slab_digest(f[slice(*slab_bounds(shape[2], n, r))]) for r in range(n)]
            out[verify.golden_key(shape, n)] = {
                "slabs": slabs, "steps": verify.CHECK_STEPS, "C": 0.0,
                "params": {k: P[k] for k in ("dtau", "m2", "lam", "seed")},
                "init": f"verify.hash_field (splitmix64, key {verify.HASH_FIELD_KEY:#x}, amp {verify.HASH_FIELD_AMP})",
                "source": "oracle/orc_phi4.c orc_phi4_step (CPU), tests/golden/make_oracle_slabs.py"}
            print(verify.golden_key(shape, n), slabs[:2], f"{time.time() - t0:.1f} s", flush=True)
        del f
    with open(verify.ORACLE_GOLDEN, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", verify.ORACLE_GOLDEN)


if __name__ == "__main__":
    main()
