"""A/B of the fused kernel's balance knobs between the two blocks a CU holds
(SQ_TB2_PRIO, SQ_TB2_PSHIFT, SQ_TB2_ZSPLIT, read from the environment): us/step over 2000
steps at 256^3, block durations by dispatch round, and a field digest after
24 steps from a fixed field (must not depend on the knobs).
    SQ_TB2_ZSPLIT=1 python scripts/ab_tb2_balance.py"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stochquant_amd import Phi4Lattice
    out = {"prio": os.environ.get("SQ_TB2_PRIO", "1"), "pshift": os.environ.get("SQ_TB2_PSHIFT", "0"), "zsplit": os.environ.get("SQ_TB2_ZSPLIT", "0")}
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as lat:
        lat.init_field(0.1)
        lat.step(24)
        lat.sync()
        out["digest"] = hashlib.sha256(lat.download().tobytes()).hexdigest()[:16]
        lat.step(1000)
        lat.sync()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            lat.step(2000)
            lat.sync()
            ts.append((time.perf_counter() - t0) * 1e6 / 2000)
        out["us_per_step"] = [round(t, 3) for t in ts]
        out["median"] = round(float(np.median(ts)), 3)
        D, E = [], []
        for _ in range(8):
            lat.step(300)
            st, en = lat.block_stamps()
            t0 = st.min()
            D.append((en - st) * 1e-2)
            E.append((en - t0) * 1e-2)
        D, E = np.array(D), np.array(E)
        nb = D.shape[1]
        r2 = np.arange(nb) * 2 >= nb
        out["dur_round1_round2_us"] = [round(float(D[:, ~r2].mean()), 2), round(float(D[:, r2].mean()), 2)]
        out["span_us"] = round(float(E.max(1).mean()), 2)
        out["busy"] = round(float((D.sum(1) / (nb * E.max(1))).mean()), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
