"""A/B of one step per launch vs the two-step fused kernel (and its register
budget / blocks per CU) on one GPU, all variants in ONE process, interleaved
rounds.  Prints one JSON line per (variant, round) and the medians.

    python scripts/sweep_tb2.py --shape 512x512x512 [--steps 200] [--rounds 3]
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
    ap.add_argument("--shape", default="512x512x512")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="fuse0;fuse1,wpe6,bpc2;fuse1,wpe1,bpc1;fuse1,wpe1,bpc2")
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice
    shape = tuple(int(v) for v in a.shape.split("x"))
    sites = shape[0] * shape[1] * shape[2]
    lats = {}
    for v in a.variants.split(";"):
        kv = dict((t[:4], t[4:]) for t in v.split(","))
        os.environ["SQ_FUSE2"] = kv.get("fuse", "1")
        os.environ["SQ_TB2_WPE"] = kv.get("wpe", "6")
        os.environ["SQ_TB2_BLOCKS_PER_CU"] = kv.get("bpc", "2")
        if "zc" in kv:
            os.environ["SQ_FUSE2_Z"] = kv["zc"]
        else:
            os.environ.pop("SQ_FUSE2_Z", None)
        lat = Phi4Lattice(shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED)
        lat.init_field(0.1)
        lat.step(50)
        lat.sync()
        lats[v] = lat
        print(v, lat.kernel_name, flush=True)
    res = {v: [] for v in lats}
    for rnd in range(a.rounds):
        for v, lat in lats.items():
            lat.perf_reset()
            lat.set_profiling(2)
            t0 = time.perf_counter()
            lat.step(a.steps)
            lat.sync()
            wall = (time.perf_counter() - t0) / a.steps * 1e6
            p = lat.perf()
            lat.set_profiling(0)
            k = p["step_kernel_ms"] / p["step_kernel_launches"] * 1e3
            res[v].append(k)
            print(json.dumps({"variant": v, "round": rnd, "us_per_step_events": round(k, 3),
                              "us_per_step_wall": round(wall, 3),
                              "alg_GBps": round(8 * sites / (k * 1e-6) / 1e9, 1)}), flush=True)
    print("summary (median us per step by events, algorithmic GB/s):")
    for v in sorted(res, key=lambda v: statistics.median(res[v])):
        k = statistics.median(res[v])
        print(f"{v:32s} {k:9.3f} us  {8 * sites / (k * 1e-6) / 1e9:8.1f} GB/s  {sites / (k * 1e-6):.4g} site-updates/s")
    for lat in lats.values():
        lat.close()


if __name__ == "__main__":
    main()
