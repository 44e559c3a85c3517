"""Per-step time of the phi^4 step vs the lattice depth Lz at fixed 256 x 256
planes (one GPU, interleaved rounds): t(Lz) = a + b Lz separates the fixed
per-launch cost (dispatch ramp, tail, kernel boundary) from the per-plane cost.

    python scripts/lz_scan.py [--lz 64,128,192,256,320] [--steps 1000] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lz", default="64,128,192,256,320")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice
    lzs = [int(v) for v in a.lz.split(",")]
    lats = {}
    for lz in lzs:
        lat = Phi4Lattice((256, 256, lz), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
        lat.init_field(0.1)
        lat.step(500)
        lat.sync()
        lats[lz] = lat
    res = {lz: [] for lz in lzs}
    for rnd in range(a.rounds):
        for lz in lzs:
            lat = lats[lz]
            t0 = time.perf_counter()
            lat.step(a.steps)
            lat.sync()
            us = (time.perf_counter() - t0) / a.steps * 1e6
            res[lz].append(us)
            print(json.dumps({"Lz": lz, "round": rnd, "wall_us_per_step": round(us, 3)}), flush=True)
    xs = lzs
    ys = [statistics.median(res[lz]) for lz in lzs]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    print(json.dumps({"fit": "t = a + b*Lz", "a_us": round(my - b * mx, 3), "b_us_per_plane": round(b, 5),
                      "medians": dict(zip(map(str, xs), [round(y, 3) for y in ys]))}), flush=True)
    for lat in lats.values():
        lat.close()


if __name__ == "__main__":
    main()
