"""Diagnostic: frames that stay stable must equal the same number of raw steps
(same noise counters); run per path (fused single slab, RCCL self-exchange)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stochquant_amd import Phi4Lattice, unique_id  # noqa: E402

shape = (256, 8, 16)
rng = np.random.default_rng(77)
phi0 = (0.9 * rng.standard_normal((shape[2], shape[1], shape[0]))).astype(np.float32)
KW = dict(dtau=0.02, m2=0.5, lam=1.0, seed=77)


def run(frames, **kw):
    with Phi4Lattice(shape, loops=6, **KW, **kw) as L:
        L.upload(phi0)
        if frames:
            for _ in range(3):
                assert L.run_frame()
        else:
            L.step(18)
        return L.download(), L.kernel_name


for name, kw, env in [("mono", {}, {}), ("rccl", None, {"SQ_GHOST": "4"})]:
    os.environ.update(env)
    k = kw if kw is not None else dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id())
    a, kn = run(True, **k)
    k = kw if kw is not None else dict(comm="rccl", nranks=1, rank=0, comm_id=unique_id())
    b, _ = run(False, **k)
    d = np.argwhere(a != b)
    print(name, kn, "frames==steps:", np.array_equal(a, b), "ndiff", len(d), d[:6].tolist(), flush=True)
    globals()[name] = (a, b)
print("mono steps == rccl steps:", np.array_equal(mono[1], rccl[1]))
print("mono frames == rccl frames:", np.array_equal(mono[0], rccl[0]))
