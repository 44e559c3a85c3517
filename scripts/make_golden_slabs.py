"""Golden slab digests for bench.py's multi_rank_check (stochquant_amd/verify.py),
from single-GPU runs of the global lattices: the weak-scaling 256 x 256 x 256N
and the strong-scaling 1024^3, N = 1, 2, 4, 8, each digest over the planes
rank r of N owns (decomp.slab_bounds).  Run on one MI355X:
    python scripts/make_golden_slabs.py [out.json]  (default stochquant_amd/golden_slabs.json)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stochquant_amd import Phi4Lattice  # noqa: E402
from stochquant_amd.decomp import slab_bounds  # noqa: E402
from stochquant_amd import verify  # noqa: E402


def main():
    out = {}
    P = verify.CHECK_PARAMS
    cases = [((256, 256, 256 * n), [n]) for n in (1, 2, 4, 8)] + [((1024, 1024, 1024), [1, 2, 4, 8])]
    for shape, ns in cases:
        with Phi4Lattice(shape, dtau=P["dtau"], m2=P["m2"], lam=P["lam"], seed=P["seed"]) as L:
            d = verify.run_protocol(L)
            f = L.download()
            kname = L.kernel_name
        for n in ns:
            slabs = [verify.slab_digest(f[slice(*slab_bounds(shape[2], n, r))]) for r in range(n)]
            out[verify.golden_key(shape, n)] = {"slabs": slabs, "steps": verify.CHECK_STEPS, "params": P,
                                                "kernel": kname}
            print(verify.golden_key(shape, n), slabs[:2], flush=True)
        assert verify.slab_digest(f) == d
        del f
    path = sys.argv[1] if len(sys.argv) > 1 else verify.GOLDEN
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
