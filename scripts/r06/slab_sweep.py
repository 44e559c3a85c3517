"""Slab-path schedule sweep on one GPU: RCCL / P2P
self-exchange of the 256^3 lattice under pinned schedule knobs (ghost depth G,
core pairs K, rims on stream B, edges-first), each against the single slab
timed right before it (bench.py's slab_record method: 400 warm-up steps, then
`steps` timed), two interleaved passes.  One JSON line per measurement."""
import json
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from stochquant_amd import Phi4Lattice, unique_id  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
KNOBS = ("SQ_GHOST", "SQ_CORE_PAIRS", "SQ_RIMS_B", "SQ_EDGE_FIRST", "SQ_XCHG_BLOCKS", "SQ_XCHG_PRIO",
         "SQ_EDGES_STOPEV")
CASES = [
    ("rccl", {}),
    ("rccl", {"SQ_GHOST": "12"}), ("rccl", {"SQ_GHOST": "20"}), ("rccl", {"SQ_GHOST": "24"}),
    ("rccl", {"SQ_GHOST": "32"}),
    ("rccl", {"SQ_GHOST": "16", "SQ_RIMS_B": "1"}),
    ("rccl", {"SQ_GHOST": "16", "SQ_EDGE_FIRST": "1"}),
    ("rccl", {"SQ_GHOST": "16", "SQ_CORE_PAIRS": "0"}),
    ("rccl", {"SQ_GHOST": "16", "SQ_CORE_PAIRS": "0", "SQ_EDGE_FIRST": "1"}),
    ("rccl", {"SQ_GHOST": "24", "SQ_CORE_PAIRS": "2"}),
    ("p2p", {}), ("p2p", {"SQ_GHOST": "24"}), ("p2p", {"SQ_GHOST": "32"}),
]
kw = dict(dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)


def timed(L):
    L.init_field(0.1)
    L.step(400)
    L.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.step(STEPS)
    L.sync()
    return (time.perf_counter() - t0) * 1e6 / STEPS


REPS = 2
if len(sys.argv) > 2 and sys.argv[2] == "p2ponly":
    CASES = [("p2p", {}), ("rccl", {}), ("p2p", {"SQ_GHOST": "24"})]
if len(sys.argv) > 2 and sys.argv[2] == "prio":
    CASES = [("rccl", {}), ("rccl", {"SQ_XCHG_PRIO": "0"}), ("rccl", {"SQ_EDGES_STOPEV": "1"}),
             ("rccl", {"SQ_GHOST": "12"}), ("p2p", {}), ("p2p", {"SQ_XCHG_PRIO": "0"}), ("p2p", {"SQ_GHOST": "12"})]
    REPS = 4
for rep in range(REPS):
    for comm, env in CASES:
        for k in KNOBS:
            os.environ.pop(k, None)
        with Phi4Lattice((256, 256, 256), **kw) as L:
            base = timed(L)
        os.environ.update(env)
        if comm == "rccl":
            L = Phi4Lattice((256, 256, 256), comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
        else:
            L = Phi4Lattice((256, 256, 256), comm="p2p", nranks=1, rank=0, **kw)
            L.p2p_connect([L.p2p_handle()])
        with L:
            us = timed(L)
            sch = L.schedule
        print(json.dumps({"rep": rep, "comm": comm, "env": env, "single_us": round(base, 3), "us": round(us, 3),
                          "ratio": round(us / base, 4), "schedule": sch}), flush=True)
for k in KNOBS:
    os.environ.pop(k, None)
