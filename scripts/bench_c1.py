"""C1 alone (the 32,768-site QM1D chain, 1000-step Jacobi frames): bench.py's
c1_qm1d sub-record without the 3-D lattices, for A/B runs of the grid kernel
(SQ_LIB picks the library).

    python scripts/bench_c1.py [--frames 16]
"""
import argparse
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    a = ap.parse_args()
    import bench
    r = bench.c1_record(types.SimpleNamespace(c1_frames=a.frames, cpu_loops_c1=0, no_cpu_baseline=True), 0)
    print(json.dumps({"ms_per_frame": round(r["ms_per_frame"], 4), "kernel_ms_per_frame": r["kernel_ms_per_frame"],
                      "value": r["value"], "stable_frames": r["stable_frames"], "frames": r["frames"]}), flush=True)


if __name__ == "__main__":
    main()
