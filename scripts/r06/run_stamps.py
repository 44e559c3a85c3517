"""Where the resident march's time goes (SQ_DIAG_RUN_STAMPS): per pair and
block the start (its neighbours' wait done) and end (stores drained) on the
100 MHz constant clock, and each block's hardware slot.  256^3, 20-step calls
(10 pairs) after a clock settle.  Prints, over the last calls: the time per
pair (span of the launch / pairs), the mean block busy time per pair, the mean
wait between a block's end of pair t and its start of pair t+1, how far the two
blocks of one CU drift apart (pairs), and, for reference, the per-pair kernel's
block durations from block_stamps.
    python scripts/r06/run_stamps.py [calls] [prio]"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from stochquant_amd import Phi4Lattice  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8
prio = sys.argv[2] if len(sys.argv) > 2 else "1"
shape = (256, 256, 256)
path = os.path.join(tempfile.mkdtemp(), "stamps.bin")
os.environ["SQ_TB2_RUN"] = "1"
os.environ["SQ_TB2_RUN_SC1"] = os.environ.get("SQ_TB2_RUN_SC1", "1")
os.environ["SQ_TB2_RUN_PRIO"] = prio
L = Phi4Lattice(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, C=1.0, device=0)
L.init_field(0.1)
t_end = time.perf_counter() + 1.0
while time.perf_counter() < t_end:
    L.step(50)
    L.sync()
os.environ["SQ_DIAG_RUN_STAMPS"] = path
for _ in range(calls):
    L.step(20)
    L.sync()
del os.environ["SQ_DIAG_RUN_STAMPS"]
raw = np.fromfile(path, dtype=np.uint64)
off, launches = 0, []
while off < raw.size:
    P, nb = int(raw[off]), int(raw[off + 1])
    n = 2 * P * nb + nb
    w = raw[off + 2: off + 2 + n].astype(np.int64)
    launches.append((P, nb, w[:2 * P * nb].reshape(P, nb, 2), raw[off + 2 + 2 * P * nb: off + 2 + n]))
    off += 2 + n
per_pair, busy, wait, drift, first = [], [], [], [], []
for P, nb, st, hw in launches[1:]:
    t0 = st[:, :, 0].min()
    span = st[:, :, 1].max() - t0
    per_pair.append(span / P / 100.0)
    busy.append(((st[:, :, 1] - st[:, :, 0]).mean()) / 100.0)
    wait.append(((st[1:, :, 0] - st[:-1, :, 1]).mean()) / 100.0)
    first.append((st[0, :, 1].max() - st[0, :, 0].min()) / 100.0)
    # the two blocks of each CU: (XCC, HW_ID bits 8-15 = CU / SH / SE)
    key = (hw.astype(np.int64) >> 16) * 256 + ((hw.astype(np.int64) >> 8) & 0xFF)
    groups = {}
    for b, k in enumerate(key):
        groups.setdefault(int(k), []).append(b)
    sizes = sorted({len(v) for v in groups.values()})
    d = []
    for v in groups.values():
        if len(v) == 2:
            a, c = v
            # at each of a's pair starts, how many pairs c has started by then
            for t in range(P):
                d.append(np.searchsorted(st[:, c, 0], st[t, a, 0], side="right") - 1 - t)
    drift.append(np.abs(np.array(d)).mean() if d else float("nan"))
print(f"launches {len(launches)}, pairs {launches[0][0]}, blocks {launches[0][1]}, CU group sizes {sizes}")
print(f"time per pair (launch span / pairs) {np.median(per_pair):.2f} us; first pair's span {np.median(first):.2f}")
print(f"block busy per pair {np.median(busy):.2f} us; wait between pairs {np.median(wait):.2f} us")
print(f"|pairs between the two blocks of a CU| mean {np.nanmedian(drift):.3f}")
os.environ["SQ_TB2_RUN"] = "0"
Q = Phi4Lattice(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, C=1.0, device=0)
Q.init_field(0.1)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    Q.step(50)
    Q.sync()
dur, span = [], []
for _ in range(8):
    Q.step(6)
    s, e = Q.block_stamps()
    dur.append((e - s).mean() / 100.0)
    span.append((e.max() - s.min()) / 100.0)
print(f"per-pair kernel (block_stamps): block duration mean {np.median(dur):.2f} us, launch span {np.median(span):.2f} us")
