"""One slab-path configuration on one GPU for a kernel trace (VERDICT r5 next
#2: the per-block budget before any change): 256^3, the same contexts as
bench.py's slab_record -- 'single' (one periodic slab), 'rccl' (RCCL
self-exchange), 'p2p' (peer-pointer self-exchange) -- 400 warm-up steps, then
`steps` steps; prints the wall us/step.  Run under rocprofv3 --kernel-trace
and read the trace with scripts/r06/slab_budget.py."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from stochquant_amd import Phi4Lattice, unique_id  # noqa: E402

name = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 320
kw = dict(dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
if name == "single":
    L = Phi4Lattice((256, 256, 256), **kw)
elif name == "rccl":
    L = Phi4Lattice((256, 256, 256), comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
else:
    L = Phi4Lattice((256, 256, 256), comm="p2p", nranks=1, rank=0, **kw)
    L.p2p_connect([L.p2p_handle()])
with L:
    L.init_field(0.1)
    L.step(400)
    L.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.step(steps)
    L.sync()
    us = (time.perf_counter() - t0) * 1e6 / steps
    print(name, "us/step", round(us, 3), "schedule", None if name == "single" else L.schedule, flush=True)
