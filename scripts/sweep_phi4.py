"""Tuning sweep of the phi^4 step kernel on one GPU, all variants in ONE
process (interleaved rounds, guide §5.4 rule 24).  Prints one JSON line per
(variant, round) and a summary of medians.

    python scripts/sweep_phi4.py [--size 256] [--steps 400] [--rounds 3]
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rows", default="1,2,4")
    ap.add_argument("--zc", default="2,4,8,16")
    ap.add_argument("--pf", default="1", help="z prefetch distances to try (1,2)")
    ap.add_argument("--vseg", default="0", help="float4 segments per lane to try (0 = library default)")
    ap.add_argument("--wpb", default="4", help="waves per block to try (needs a build with SQ_WPB; "
                                               "measured no gain, profiles/r01/sweep*_wpb.log)")
    ap.add_argument("--C", type=float, default=1.0, help="noise amplitude (0: RNG-free gradient-flow kernel)")
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice
    L = a.size
    variants = list(itertools.product([int(r) for r in a.rows.split(",")], [int(z) for z in a.zc.split(",")],
                                      [int(p) for p in a.pf.split(",")], [int(v) for v in a.vseg.split(",")],
                                      [int(w) for w in a.wpb.split(",")]))
    res = {v: [] for v in variants}
    lats = {}
    for v in variants:
        os.environ["SQ_ROWS"], os.environ["SQ_ZCHUNK"], os.environ["SQ_PREFETCH"] = str(v[0]), str(v[1]), str(v[2])
        os.environ["SQ_WPB"] = str(v[4])
        if v[3]:
            os.environ["SQ_VSEG"] = str(v[3])
        else:
            os.environ.pop("SQ_VSEG", None)
        lat = Phi4Lattice((L, L, L), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, C=a.C)
        lat.init_field(0.1)
        lat.step(50)
        lat.sync()
        lats[v] = lat
    for rnd in range(a.rounds):
        for v in variants:
            lat = lats[v]
            row = {"rows": v[0], "zc": v[1], "pf": v[2], "vseg": v[3], "wpb": v[4], "round": rnd}
            for mode in (0, 1, 2):
                lat.perf_reset()
                lat.set_profiling(mode)
                t0 = time.perf_counter()
                lat.step(a.steps)
                lat.sync()
                wall = (time.perf_counter() - t0) / a.steps * 1e6
                p = lat.perf()
                lat.set_profiling(0)
                row[f"wall_us_m{mode}"] = round(wall, 3)
                if mode:
                    row[f"kernel_us_m{mode}"] = round(p["step_kernel_ms"] / p["step_kernel_launches"] * 1e3, 3)
            res[v].append((row["kernel_us_m1"], row["wall_us_m0"]))
            row["GBps_m1"] = round(8 * L ** 3 / (row["kernel_us_m1"] * 1e-6) / 1e9, 1)
            print(json.dumps(row), flush=True)
    print("summary (median per-launch kernel us [mode 1], median un-instrumented wall us/step, GB/s by kernel):")
    for v in sorted(variants, key=lambda v: statistics.median(k for k, _ in res[v])):
        k = statistics.median(x for x, _ in res[v])
        w = statistics.median(y for _, y in res[v])
        print(f"rows={v[0]} zc={v[1]:3d} pf={v[2]} v={v[3]} wpb={v[4]}  kernel {k:8.3f} us  wall {w:8.3f} us  {8 * L ** 3 / (k * 1e-6) / 1e9:8.1f} GB/s")
    for lat in lats.values():
        lat.close()


if __name__ == "__main__":
    main()
