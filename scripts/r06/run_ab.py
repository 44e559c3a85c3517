"""A/B of the resident two-step march (SQ_TB2_RUN=1) against one launch per
pair at 256^3, in one process: three contexts (pair launches, march with an
acquire per pair, march with sc1 loads), rotated order, several rounds.  Each
round times, per context, the driver's headline shape (one sq_step(20) call,
wall clock from an idle device, as bench.py's timed region) R times, and a
2000-step call (steady state).  Prints medians per context.
    python scripts/r06/run_ab.py [rounds]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from stochquant_amd import Phi4Lattice  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
shape = (256, 256, 256)
sites = shape[0] * shape[1] * shape[2]
# name: (SQ_TB2_RUN, SQ_TB2_RUN_SC1, SQ_TB2_RUN_PRIO, SQ_TB2_RUN_MAXP)
cfg = {"pairs": ("0", "0", "1", "0"), "run_sc1": ("1", "1", "1", "0"), "run_sc1_noprio": ("1", "1", "0", "0")}
mode = sys.argv[2] if len(sys.argv) > 2 else ""
if mode == "acq":
    cfg = {"pairs": ("0", "0", "1", "0"), "run_acq": ("1", "0", "1", "0"), "run_acq_noprio": ("1", "0", "0", "0")}
elif mode == "maxp":  # one pair per resident launch: the hand-off's own cost without the dataflow
    cfg = {"pairs": ("0", "0", "1", "0"), "run_sc1": ("1", "1", "1", "0"), "run_sc1_maxp1": ("1", "1", "1", "1")}
elif mode == "maxp_acq":
    cfg = {"pairs": ("0", "0", "1", "0"), "run_acq": ("1", "0", "1", "0"), "run_acq_maxp1": ("1", "0", "1", "1")}


def setenv(n):
    os.environ["SQ_TB2_RUN_SC1"] = cfg[n][1]
    os.environ["SQ_TB2_RUN_PRIO"] = cfg[n][2]
    if cfg[n][3] != "0":
        os.environ["SQ_TB2_RUN_MAXP"] = cfg[n][3]
    else:
        os.environ.pop("SQ_TB2_RUN_MAXP", None)


ctx = {}
for name, (run, _, _, _) in cfg.items():
    os.environ["SQ_TB2_RUN"] = run
    L = Phi4Lattice(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, C=1.0, device=0)
    L.init_field(0.1)
    ctx[name] = L
names = list(cfg)
res = {n: {"w20": [], "s2000": []} for n in names}


def timed(L, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L.step(steps)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


for r in range(rounds):
    order = names[r % 3:] + names[:r % 3]
    for n in order:
        L = ctx[n]
        setenv(n)
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:  # clock settle on this context
            L.step(50)
            L.sync()
        L.step(6)
        for _ in range(10):
            res[n]["w20"].append(timed(L, 20) / 20 * 1e6)
        res[n]["s2000"].append(timed(L, 2000) / 2000 * 1e6)
        info = L.launch_info()
    print(f"round {r}: " + "  ".join(f"{n} w20 {statistics.median(res[n]['w20'][-10:]):.3f} "
                                     f"s2000 {res[n]['s2000'][-1]:.3f}" for n in names), flush=True)
for n in names:
    w, s = statistics.median(res[n]["w20"]), statistics.median(res[n]["s2000"])
    print(f"{n}: us/step 20-step call median {w:.3f} ({sites / w * 1e6:.4e} site-updates/s), "
          f"2000-step call median {s:.3f} ({sites / s * 1e6:.4e})")
for n in names:
    L = ctx[n]
    L.perf_reset()
    setenv(n)
    L.step(20)
    L.sync()
    print(n, L.launch_info())
    L.close()
