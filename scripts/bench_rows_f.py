"""Measurements of SURVEY.md §8(f) rows 1-3 on the 256^3 phi^4 lattice (one
GPU): what a frame costs on top of its raw steps (snapshot, the frame
instances of the kernels with the guard flag and stability records, the
reductions, the rule, the controller -- row 1), the observables (moments and
the zero-momentum slice correlator -- row 2), and the binary checkpoint
(row 3).  One JSON line per quantity; run under rocprofv3 --kernel-trace
--stats for the per-kernel times.

    python scripts/bench_rows_f.py [--size 256] [--loops 20] [--reps 20]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, sync):
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--loops", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from stochquant_amd import Phi4Lattice
    L = a.size
    sites = L ** 3
    fbytes = 4 * sites
    with Phi4Lattice((L, L, L), dtau=0.01, m2=1.0, lam=1.0, loops=a.loops) as lat:
        lat.init_field(0.1)
        lat.step(2000)          # clock settle
        lat.sync()
        raw = timed(lambda: lat.step(a.loops), a.reps, lat.sync)
        frame = timed(lambda: lat.run_frame(), a.reps, lat.sync)
        batch = timed(lambda: lat.run_frames(100), 3, lat.sync) / 100
        os.environ["SQ_FRAME_HOST"] = "1"
        host = timed(lambda: lat.run_frame(), a.reps, lat.sync)
        del os.environ["SQ_FRAME_HOST"]
        print(json.dumps({"row": "f1 frame control", "loops": a.loops, "raw_steps_us": round(raw * 1e6, 1),
                          "frame_us": round(frame * 1e6, 1), "overhead_us_per_frame": round((frame - raw) * 1e6, 1),
                          "overhead_frac": round(frame / raw - 1, 4),
                          "batch_frame_us": round(batch * 1e6, 1),
                          "batch_overhead_us_per_frame": round((batch - raw) * 1e6, 1),
                          "batch_overhead_frac": round(batch / raw - 1, 4),
                          "host_decided_frame_us": round(host * 1e6, 1),
                          "note": "frame: sq_run_frame (device controller, one sync per frame); batch: "
                                  "sq_run_frames(100) per frame; host_decided: SQ_FRAME_HOST=1"}), flush=True)
        mom = timed(lambda: lat.moments(), a.reps, lat.sync)
        cor = timed(lambda: lat.correlator(), a.reps, lat.sync)
        print(json.dumps({"row": "f2 observables", "moments_us": round(mom * 1e6, 1),
                          "moments_GBps_incl_host": round(fbytes / mom / 1e9, 1),
                          "correlator_us": round(cor * 1e6, 1),
                          "correlator_GBps_incl_host": round(fbytes / cor / 1e9, 1),
                          "note": "wall time per call incl. the host round trip; kernel times in the rocprofv3 stats"}),
              flush=True)
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            path = os.path.join(d, "phi.npy")
            save = timed(lambda: lat.save(path), 3, lat.sync)
            load = timed(lambda: lat.load(path), 3, lat.sync)
        print(json.dumps({"row": "f3 checkpoint", "bytes": fbytes, "save_ms": round(save * 1e3, 2),
                          "save_GBps": round(fbytes / save / 1e9, 2), "load_ms": round(load * 1e3, 2),
                          "load_GBps": round(fbytes / load / 1e9, 2),
                          "note": "D2H/H2D + .npy write/read on the box's /tmp"}), flush=True)


if __name__ == "__main__":
    main()
