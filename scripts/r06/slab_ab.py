"""Interleaved A/B of slab-path contexts on one GPU.  Every
context stays open: the single periodic slab and each slab variant (RCCL /
P2P self-exchange under the env knobs given, read at context creation); each
is warmed with 2000 steps, then ROUNDS rounds time `steps` steps of every
context in turn.  Prints per context the median us/step and its ratio to the
single slab's median -- the same quantity as bench.py's slab_record, without
its single-measurement clock noise.

    python scripts/r06/slab_ab.py STEPS ROUNDS name:comm[:K=V,...] ...
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from stochquant_amd import Phi4Lattice, unique_id  # noqa: E402

steps, rounds = int(sys.argv[1]), int(sys.argv[2])
kw = dict(dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
ctxs = {"single": Phi4Lattice((256, 256, 256), **kw)}
for spec in sys.argv[3:]:
    name, comm, *rest = spec.split(":")
    env = dict(kv.split("=") for kv in rest[0].split(",")) if rest and rest[0] else {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    if comm == "rccl":
        L = Phi4Lattice((256, 256, 256), comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
    else:
        L = Phi4Lattice((256, 256, 256), comm="p2p", nranks=1, rank=0, **kw)
        L.p2p_connect([L.p2p_handle()])
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    ctxs[name] = L
for L in ctxs.values():
    L.init_field(0.1)
    L.step(2000)
    L.sync()
times = {n: [] for n in ctxs}
for r in range(rounds):
    for n, L in ctxs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.step(steps)
        L.sync()
        times[n].append((time.perf_counter() - t0) * 1e6 / steps)
base = statistics.median(times["single"])
out = {}
for n, v in times.items():
    m = statistics.median(v)
    out[n] = {"median_us": round(m, 3), "ratio": round(m / base, 4), "min_us": round(min(v), 3),
              "schedule": ctxs[n].schedule if n != "single" else None}
print(json.dumps({"steps": steps, "rounds": rounds, "contexts": out}), flush=True)
for L in ctxs.values():
    L.close()
