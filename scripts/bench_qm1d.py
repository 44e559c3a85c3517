"""QM1D frame time on the GPU vs the oracle on one host core, for the
reference's preset shapes and config C1's 32,768-site chain.

    python scripts/bench_qm1d.py [--frames 5] [--ordering serial|jacobi]

serial: SQ_ORDER_SERIAL vs the serial oracle (orc_serial_launch);
jacobi: the default Jacobi/Philox frame vs the Jacobi oracle (orc_qm1d_frame).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--ordering", default="serial", choices=["serial", "jacobi"])
    ap.add_argument("--no-cpu", action="store_true", help="GPU timings only (no oracle run)")
    ap.add_argument("--no-c1", action="store_true", help="skip config C1's 32,768-site chain")
    a = ap.parse_args()
    import oracle
    from stochquant_amd import Qm1dChain
    # (N, dt, dtau, potID, loops): taumain.py presets' shapes and the C1-like chain
    shapes = [(100, 0.1, 0.002, 3, 1000), (200, 0.1, 0.002, 3, 200), (1000, 0.05, 0.0005, 0, 1000),
              (3072, 0.05, 0.0005, 0, 200)]
    if a.ordering == "jacobi" and not a.no_c1:
        shapes.append((32768, 1.0, 0.01, 0, 1000))  # config C1
    for N, dt, dtau, pot, loops in shapes:
        f0 = 0.1 * np.random.default_rng(1).standard_normal(N)
        kw = dict(ordering="serial", lcg_seed=12345) if a.ordering == "serial" else {}
        with Qm1dChain(N, dt, dtau, pot=pot, C=1.0, loops=loops, **kw) as g:
            g.upload(f0, omega=dt * (N // 2))
            g.run_frame()  # warm-up (allocations, code objects)
            g.sync()
            t0 = time.perf_counter()
            st = [g.run_frame() for _ in range(a.frames)]
            g.sync()
            gpu_ms = (time.perf_counter() - t0) * 1e3 / a.frames
        if a.no_cpu:
            print(json.dumps({"ordering": a.ordering, "N": N, "loops": loops, "pot": pot, "stable_frames": int(sum(st)),
                              "gpu_ms_per_frame": round(gpu_ms, 3), "qm1d_k": os.environ.get("SQ_QM1D_K")}), flush=True)
            continue
        nf = max(1, min(a.frames, int(2e6 // (N * loops)) or 1))
        if a.ordering == "serial":
            ch = oracle.SerialChain(N, dt, dtau, pot, 1.0, loops, 12345, f0, omega=dt * (N // 2))
            t0 = time.perf_counter()
            for _ in range(nf):
                ch.frame()
        else:
            t0 = time.perf_counter()
            for k in range(nf):
                oracle.qm1d_frame(N, dt, dtau, pot, 1.0, loops, 0x5EED, k * loops, 0, f0, np.zeros(N), np.zeros(N),
                                  dt * (N // 2))
        cpu_ms = (time.perf_counter() - t0) * 1e3 / nf
        print(json.dumps({"ordering": a.ordering, "N": N, "loops": loops, "pot": pot, "stable_frames": int(sum(st)),
                          "gpu_ms_per_frame": round(gpu_ms, 3), "cpu_oracle_ms_per_frame": round(cpu_ms, 3),
                          "gpu_site_updates_per_s": N * loops / gpu_ms * 1e3,
                          "cpu_site_updates_per_s": N * loops / cpu_ms * 1e3}), flush=True)


if __name__ == "__main__":
    main()
