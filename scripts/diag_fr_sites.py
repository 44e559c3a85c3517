"""Which sites does a frame launch get wrong?  One frame of `loops` steps vs the
same raw steps, repeated; prints the differing sites (z, y, x), their lanes
(x // 4) and planes.  argv: loops C pre_steps reps"""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stochquant_amd import Phi4Lattice  # noqa: E402

loops, C, pre, reps = (int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
shape = tuple(int(v) for v in os.environ.get("DIAG_SHAPE", "256,8,16").split(","))
rng = np.random.default_rng(77)
phi0 = (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)
KW = dict(dtau=0.02, m2=0.5, lam=1.0, seed=77, C=C)


def run(frames):
    with Phi4Lattice(shape, loops=loops, **KW) as L:
        L.upload(phi0)
        if pre:
            L.step(pre)
        if frames:
            assert L.run_frame()
        else:
            L.step(loops)
        return L.download()


ref = run(False)
for r in range(reps):
    got = run(True)
    d = np.argwhere(got != ref)
    lanes = sorted(set((int(x) // 4) for x in d[:, 2])) if len(d) else []
    planes = sorted(set(int(z) for z in d[:, 0])) if len(d) else []
    rows = sorted(set(int(y) for y in d[:, 1])) if len(d) else []
    print(f"loops={loops} C={C} pre={pre} rep {r}: ndiff {len(d)} planes {planes[:20]} rows {rows[:20]} "
          f"lanes {lanes[:40]}", flush=True)
    if len(d):
        print("   first:", d[:12].tolist(), flush=True)
        k = tuple(d[0])
        print("   got", got[k], "ref", ref[k], flush=True)
