"""Frames that stay stable must equal the same raw steps on the same noise
counters (scripts/diag_frame_vs_steps.py), repeated, over shapes and paths,
for whichever fused kernel SQ_TB2_PIPE selects.  Prints one line per case."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stochquant_amd import Phi4Lattice, unique_id  # noqa: E402

KW = dict(dtau=0.02, m2=0.5, lam=1.0, seed=77)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3


def run(shape, phi0, frames, rccl):
    kw = dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id()) if rccl else {}
    with Phi4Lattice(shape, loops=6, **KW, **kw) as L:
        L.upload(phi0)
        if frames:
            for _ in range(3):
                assert L.run_frame()
        else:
            L.step(18)
        return L.download(), L.kernel_name


bad = 0
for shape in [(256, 8, 16), (256, 16, 24), (512, 8, 16), (256, 64, 64)]:
    rng = np.random.default_rng(77)
    phi0 = (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)
    for rccl in (False, True):
        if rccl:
            os.environ["SQ_GHOST"] = "4"
        ref, kn = run(shape, phi0, False, rccl)
        for r in range(reps):
            got, _ = run(shape, phi0, True, rccl)
            d = np.argwhere(got != ref)
            bad += len(d) > 0
            print(shape, "rccl" if rccl else "mono", "rep", r, "frames==steps:", len(d) == 0, "ndiff", len(d),
                  d[:4].tolist(), kn[:30], flush=True)
        os.environ.pop("SQ_GHOST", None)
print("FAILED CASES:", bad)
