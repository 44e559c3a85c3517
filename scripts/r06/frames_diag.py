"""Where does the frames_256 overhead come from?  256^3,
20-step frames, batches of 100 through sq_run_frames, against raw 20-step
blocks, four ways:
  plain       frames then raw (bench.py's frames_record order)
  raw_first   raw then frames
  queued      frames enqueued behind 2000 queued raw steps (the host is then
              68 ms ahead: a host-bound frame loop would show its GPU-only time)
  alternate   5 x (raw 400 steps, 20 frames) interleaved, summed per kind
Prints one JSON line per way with us per frame, us per 20 raw steps and the
overhead."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from stochquant_amd import Phi4Lattice  # noqa: E402

NF, LOOPS = 100, 20


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, loops=LOOPS) as L:
    L.init_field(0.1)
    L.run_frames(20)
    L.step(200)
    L.sync()
    for rep in range(2):
        tf = wall(lambda: L.run_frames(NF))
        L.step(400)
        tr = wall(lambda: L.step(NF * LOOPS))
        print(json.dumps({"way": "plain", "rep": rep, "us_frame": tf * 1e6 / NF, "us_raw20": tr * 1e6 / NF,
                          "overhead": tf / tr - 1}), flush=True)
        tr = wall(lambda: L.step(NF * LOOPS))
        tf = wall(lambda: L.run_frames(NF))
        print(json.dumps({"way": "raw_first", "rep": rep, "us_frame": tf * 1e6 / NF, "us_raw20": tr * 1e6 / NF,
                          "overhead": tf / tr - 1}), flush=True)
        t_raw = wall(lambda: L.step(2 * NF * LOOPS))
        t_both = wall(lambda: (L.step(2 * NF * LOOPS), L.run_frames(NF)))
        tq = t_both - t_raw
        print(json.dumps({"way": "queued", "rep": rep, "us_frame": tq * 1e6 / NF,
                          "us_raw20": t_raw * 1e6 / (2 * NF), "overhead": tq / (t_raw / 2) - 1}), flush=True)
        sf = sr = 0.0
        for _ in range(5):
            sr += wall(lambda: L.step(20 * LOOPS))
            sf += wall(lambda: L.run_frames(20))
        print(json.dumps({"way": "alternate", "rep": rep, "us_frame": sf * 1e6 / 100, "us_raw20": sr * 1e6 / 100,
                          "overhead": sf / sr - 1}), flush=True)
