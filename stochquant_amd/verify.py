"""Self-check of a (multi-rank) φ⁴ run against golden slab digests.

A slab decomposition is bit-identical to the single-slab run of the same
global lattice (the noise is keyed by global site and step), so
after a fixed check protocol -- the bench's initial field (0.1·Philox normal,
seed 0x5EED), the step counter reset to 0, CHECK_STEPS steps at Δτ = 0.01,
m² = λ = 1 -- every rank's slab must hash to the digest of the same planes of
a single-GPU run.  `golden_slabs.json` holds those digests, made on one MI355X
by scripts/make_golden_slabs.py for the bench's weak-scaling lattices
256 × 256 × 256N and the strong-scaling 1024³, N = 1, 2, 4, 8.

bench.py runs the protocol after its timed region on every rank, gathers the
digests and prints "multi_rank_check": "pass" / "fail" (or "no golden").
"""
import hashlib
import json
import os

import numpy as np

CHECK_STEPS = 24          # more than one deep-halo block at any ghost depth <= 16: two exchanges
CHECK_PARAMS = dict(dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, amp=0.1)
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_slabs.json")


def slab_digest(field):
    """blake2b-128 of the slab's fp32 bytes (C order, z slowest)."""
    a = np.ascontiguousarray(field, dtype=np.float32)
    return hashlib.blake2b(a.tobytes(), digest_size=16).hexdigest()


def golden_key(shape, nranks):
    return f"{shape[0]}x{shape[1]}x{shape[2]}/{nranks}"


def load_golden(path=GOLDEN):
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def check(digests, shape, nranks, golden=None):
    """'pass' when every rank's digest equals the golden one of its slab,
    'fail' when any differs, 'no golden' when the lattice has none."""
    g = (load_golden() if golden is None else golden).get(golden_key(shape, nranks))
    if g is None:
        return "no golden"
    if len(digests) != nranks or len(g["slabs"]) != nranks:
        return "fail"
    return "pass" if all(d == e for d, e in zip(digests, g["slabs"])) else "fail"


def run_protocol(lat, corrupt=False):
    """Run the check protocol on an open Phi4Lattice (collective in multi-rank
    contexts) and return this rank's slab digest.  corrupt: flip one value of
    the slab before hashing (tests the checker itself)."""
    lat.init_field(CHECK_PARAMS["amp"])
    lat.step_counter = 0
    lat.step(CHECK_STEPS)
    f = lat.download()
    if corrupt:
        f = f.copy()
        f.flat[f.size // 2] += np.float32(1.0)
    return slab_digest(f)
