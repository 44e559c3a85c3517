"""Oracle digests for bench.py's `oracle_check` (stochquant_amd/verify.py) --
test infrastructure: runs the CPU oracle (oracle/orc_phi4.c, the reference's
per-site update tau_kernel.cl:111-117 restated for the 3-D φ⁴ lattice) with
the noise off on the bench's lattices and writes, per rank count N, the
blake2b digest of every rank's slab after verify.CHECK_STEPS steps from
verify.hash_field.  No GPU is involved: these are the oracle's bits, which
the GPU must reproduce exactly (C = 0 is deterministic fp32 arithmetic).

Lattices: the weak-scaling 256 x 256 x 256N (N = 1, 2, 4, 8; every rank a
256^3 slab) and the strong-scaling 1024^3 (N = 1, 2, 4, 8).

    python tests/golden/make_oracle_slabs.py [--threads T] [--quick] [--noise]

(--quick: the weak lattices only.)  Output: tests/golden/oracle_slabs.json.

--noise (bench.py's `oracle_check_noise`): the same
lattices and steps with C = 1, the oracle in device-transcendental mode.  The
Box-Muller factors are tabulated on the GPU once (sq_selftest_bm_tables, so
this mode needs a device -- run it on the GPU box); the digests are stored
under "noise:<key>" beside the blake2b digest of those tables ("bm_tables"),
and the bench compares a rank's digest only when its device's tables hash the
same.  Everything else -- Philox words, the step arithmetic -- is the CPU
oracle's.
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


def oracle_run(shape, threads, C=0.0):
    P = verify.CHECK_PARAMS
    p = oracle.phi4_params(shape, P["dtau"], P["m2"], P["lam"], P["seed"], C=C)
    phi = verify.hash_field(shape, 0, shape[2])
    for s in range(verify.CHECK_STEPS):
        phi = oracle.phi4_step(p, phi, s, threads)
    return phi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--noise", action="store_true")
    ap.add_argument("--out", default=None, help="write here instead of tests/golden/oracle_slabs.json")
    a = ap.parse_args()
    oracle.build()
    out = verify.load_oracle_golden()
    if a.noise:
        return noise_digests(a, out)
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
    path = a.out or verify.ORACLE_GOLDEN
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", path)


def noise_digests(a, out):
    import contextlib
    tables = verify.bm_tables(0)
    tdig = verify.bm_tables_digest(tables)
    if out.get(verify.BM_TABLES_KEY, {}).get("blake2b") not in (None, tdig):
        # other tables: the committed noise digests no longer describe them
        for k in [k for k in out if k.startswith(verify.NOISE_PREFIX)]:
            del out[k]
    out[verify.BM_TABLES_KEY] = {
        "blake2b": tdig, "count": int(tables.size),
        "source": "sq_selftest_bm_tables on the MI355X (v_log_f32 / v_sqrt_f32 radius, v_cos_f32 / v_sin_f32 of "
                  "t revolutions, every 23-bit argument), blake2b-128 of the float32 bytes"}
    cases = [((256, 256, 256 * n), [n]) for n in (1, 2, 4, 8)]
    if not a.quick:
        cases.append(((1024, 1024, 1024), [1, 2, 4, 8]))
    P = verify.CHECK_PARAMS
    with contextlib.ExitStack() as st:
        st.enter_context(oracle.device_transcendentals(tables))
        for shape, ns in cases:
            t0 = time.time()
            f = oracle_run(shape, a.threads, C=1.0)
            for n in ns:
                slabs = [verify.slab_digest(f[slice(*slab_bounds(shape[2], n, r))]) for r in range(n)]
                out[verify.NOISE_PREFIX + verify.golden_key(shape, n)] = {
                    "slabs": slabs, "steps": verify.CHECK_STEPS, "C": 1.0, "bm_tables": tdig,
                    "params": {k: P[k] for k in ("dtau", "m2", "lam", "seed")},
                    "init": f"verify.hash_field (splitmix64, key {verify.HASH_FIELD_KEY:#x}, "
                            f"amp {verify.HASH_FIELD_AMP})",
                    "source": "oracle/orc_phi4.c orc_phi4_step (CPU) in device-transcendental mode "
                              "(oracle.device_transcendentals), tests/golden/make_oracle_slabs.py --noise"}
                print("noise:" + verify.golden_key(shape, n), slabs[:2], f"{time.time() - t0:.1f} s", flush=True)
            del f
    path = a.out or verify.ORACLE_GOLDEN
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", path, "tables", tdig)


if __name__ == "__main__":
    main()
