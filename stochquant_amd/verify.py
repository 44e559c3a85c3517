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


ORACLE_GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "oracle_slabs.json")
HASH_FIELD_KEY = 0x5EED5EED
HASH_FIELD_AMP = 0.25


def hash_field(shape, z0, nz, chunk=16):
    """The oracle check's initial field: planes [z0, z0 + nz) of a global
    (Lx, Ly, Lz) lattice, numpy order (z, y, x), float32.  Site i (global
    index (z Ly + y) Lx + x) gets splitmix64(i ^ key)'s top 24 bits as a
    uniform value in [-AMP, AMP): integer arithmetic and one exact scaling,
    identical on every host, so each rank builds its own slab and the oracle
    the whole lattice without a device RNG in between."""
    Lx, Ly, _ = shape
    out = np.empty((nz, Ly, Lx), dtype=np.float32)
    plane = Lx * Ly
    for c0 in range(0, nz, chunk):
        c1 = min(nz, c0 + chunk)
        i = np.arange((z0 + c0) * plane, (z0 + c1) * plane, dtype=np.uint64) ^ np.uint64(HASH_FIELD_KEY)
        # splitmix64 finaliser (wrapping uint64 arithmetic)
        i = i + np.uint64(0x9E3779B97F4A7C15)
        i = (i ^ (i >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        i = (i ^ (i >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        i = i ^ (i >> np.uint64(31))
        u = (i >> np.uint64(40)).astype(np.float64)          # [0, 2^24)
        out[c0:c1] = ((u - 8388608.0) * (HASH_FIELD_AMP / 8388608.0)).reshape(c1 - c0, Ly, Lx)
    return out


def load_oracle_golden(path=ORACLE_GOLDEN):
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def run_oracle_protocol(lat, corrupt=False, noise=False):
    """The parity protocol (collective in multi-rank contexts): C = 0 (noise
    False) or C = 1 (noise True), this rank's slab of hash_field
    (sq_init_field_hash, on the device), the step counter at 0, CHECK_STEPS
    steps; returns the slab digest.  With the noise off the step is
    deterministic fp32 arithmetic, so the digest must equal the oracle's
    (oracle/orc_phi4.c, tests/golden/make_oracle_slabs.py) bit for bit.  With
    it on the field is finite and inside the clamp, so the steps run the
    timed instance (the noise path with the guard's fast path) and the digest
    must equal the oracle's in device-transcendental mode: the same Philox
    words, each Box-Muller factor the device's (sq_selftest_bm_tables) --
    oracle_check_noise also compares those tables' digest."""
    C0 = float(lat.params.C)
    lat.set_noise(1.0 if noise else 0.0)
    try:
        lat.init_field_hash(HASH_FIELD_AMP, HASH_FIELD_KEY)   # = hash_field, generated on the device
        lat.step_counter = 0
        lat.step(CHECK_STEPS)
        f = lat.download()
        if corrupt:
            f.flat[f.size // 2] += np.float32(1.0)
        return slab_digest(f)
    finally:
        lat.set_noise(C0)


def oracle_check(digests, shape, nranks, golden=None, noise=False):
    """'pass' / 'fail' / 'no golden' of the protocol's digests against the oracle's."""
    key = golden_key(shape, nranks)
    g = (load_oracle_golden() if golden is None else golden).get(NOISE_PREFIX + key if noise else key)
    if g is None:
        return "no golden"
    if len(digests) != nranks or len(g["slabs"]) != nranks:
        return "fail"
    return "pass" if all(d == e for d, e in zip(digests, g["slabs"])) else "fail"


NOISE_PREFIX = "noise:"      # oracle_slabs.json keys of the C = 1 digests
BM_TABLES_KEY = "bm_tables"  # ... and the digest of the device tables they were made with


def bm_tables(device=0):
    """The device's Box-Muller factors (sq_selftest_bm_tables): 4 x 2^23 float32."""
    import ctypes
    from . import _lib
    t = np.empty(4 << 23, np.float32)
    _lib.call("sq_selftest_bm_tables", int(device), t.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return t


def bm_tables_digest(tables):
    return hashlib.blake2b(np.ascontiguousarray(tables, dtype=np.float32).tobytes(), digest_size=16).hexdigest()


def oracle_check_noise(digests, table_digests, shape, nranks, golden=None):
    """The C = 1 protocol's verdict: 'no golden' without committed digests for
    this lattice, 'tables differ' when any rank's device tables are not the
    ones the oracle digests were made with (no comparison then), else 'pass' /
    'fail'."""
    g = load_oracle_golden() if golden is None else golden
    want = g.get(BM_TABLES_KEY, {}).get("blake2b")
    if g.get(NOISE_PREFIX + golden_key(shape, nranks)) is None or want is None:
        return "no golden"
    if any(t != want for t in table_digests):
        return "tables differ"
    return oracle_check(digests, shape, nranks, golden=g, noise=True)


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
