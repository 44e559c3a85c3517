"""bench.py -- lattice-site Langevin updates/s of the 3-D φ⁴ fp32 step on MI355X.

Workload (BASELINE.json configs[1]): a 256^3 fp32 lattice
PER GPU, periodic, Δτ = 0.01, m² = 1, λ = 1, φ₀ = 0.1·normal; one "step" = one
Langevin update of every site (sq_step).  N = 1: one GPU, one HIP stream, z
wraps in-kernel.  N > 1 (launched by torch.distributed.run, one process per
GPU): weak scaling, global lattice 256 x 256 x (256 N) cut into z-slabs, halo
planes exchanged over RCCL (xGMI) on a second stream, overlapped with the
interior planes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size L]

Prints ONE JSON line (rank 0).  `value` = all site updates of all ranks / max
over ranks of the barrier-bracketed wall time of the K timed steps.
`roofline.achieved` = 8 algorithmic bytes per site update x the
site updates of one launch / mean duration of the launches in the timed
region (hipEvents recorded on the kernel's own stream by libstochquant.so).
At N = 1 on 256-wide lattices a launch fuses two steps (phi4_tb2_kernel), so
it moves the field once per two updates: `hbm_min_GBps` is the rate of that
one read + one write, `traffic` the PMC-measured bytes per launch.  `cpu_baseline` = the oracle's C port
of the same step (OpenMP over the box's host cores) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy peak reported beside it
BYTES_PER_SITE = 8              # read phi + write phi' (fp32), SURVEY.md §8d
METRIC = "lattice-site Langevin updates/sec at 256³ fp32; achieved HBM GB/s vs peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=2000,
                    help="untimed steps first (clocks settle: 2000 vs 200 measured +2.8 %%, profiles/r01/warmup_ab.log)")
    ap.add_argument("--size", type=int, default=256, help="per-GPU lattice edge (default 256 = config C2)")
    ap.add_argument("--dtau", type=float, default=0.01)
    ap.add_argument("--comm", choices=["auto", "rccl", "loopback"], default="auto",
                    help="auto: one slab at N=1, RCCL slabs at N>1; rccl/loopback force the slab path "
                         "at N=1 (RCCL self-exchange / --slabs slabs on one GPU) to exercise it")
    ap.add_argument("--slabs", type=int, default=2)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (config C5): the --size^3 lattice is split over the N GPUs "
                         "instead of --size^3 per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of the CPU sample")
    ap.add_argument("--no-profile-events", action="store_true",
                    help="no hipEvents in the timed region (roofline.achieved then uses wall time)")
    return ap.parse_args()


def cpu_baseline(L, dtau, target_s):
    """Oracle (C port of the same step, OpenMP) on a bounded sample of the workload."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/baseline infrastructure only: timed as the CPU baseline, never as the product
    oracle.build()
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    shape = (L, L, L)
    p = oracle.phi4_params(shape, dtau, 1.0, 1.0, 0x5EED)
    phi = oracle.phi4_init(p, 0.1)
    t0 = time.perf_counter()
    phi = oracle.phi4_step(p, phi, 0, cores)          # one step to size the sample
    t1 = time.perf_counter() - t0
    n = max(1, min(5000, int(target_s / max(t1, 1e-6))))
    t0 = time.perf_counter()
    for s in range(n):
        phi = oracle.phi4_step(p, phi, 1 + s, cores)
    dt = time.perf_counter() - t0
    return {"value": float(L ** 3 * n / dt), "unit": "site-updates/s", "cores": cores, "kind": "port",
            "sample": f"{n} steps of the {L}^3 fp32 phi^4 Langevin step (oracle/orc_phi4.c, OpenMP, "
                      f"{cores} threads), {dt:.2f} s"}


def pmc_traffic(L, nranks, kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if it matches this workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    same_kernel = ("phi4_tb2_kernel" in d.get("kernel", "")) == ("phi4_tb2_kernel" in kernel)
    if d.get("size") == L and d.get("nranks", 1) == nranks and same_kernel:
        return d.get("hbm_bytes_per_launch")
    return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        if world == 1 and a.gpus > 1:
            sys.exit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
        a.gpus = world
    import torch
    import torch.distributed as dist
    from stochquant_amd import Phi4Lattice, unique_id, _lib
    _lib.load()  # fail loudly if the HIP library is missing
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one node by contract: RCCL's bootstrap over loopback (data moves over xGMI)
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    L = a.size
    shape = (L, L, L) if a.strong else (L, L, L * world)
    kw = dict(dtau=a.dtau, m2=1.0, lam=1.0, seed=0x5EED, device=local)
    if world > 1:
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        lat = Phi4Lattice(shape, comm="rccl", nranks=world, rank=rank, comm_id=obj[0], **kw)
    elif a.comm == "rccl":
        lat = Phi4Lattice(shape, comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
    elif a.comm == "loopback":
        lat = Phi4Lattice(shape, comm="loopback", nslabs=a.slabs, **kw)
    else:
        lat = Phi4Lattice(shape, **kw)
    slab_path = world > 1 or a.comm != "auto"
    lat.init_field(0.1)

    def barrier():
        if world > 1:
            dist.barrier()

    if slab_path:
        lat.step(84)   # setup: the ghost-depth trial blocks (3 x (4 + 8 + 16) steps) when autotuning
    lat.step(a.warmup)
    lat.sync()
    torch.cuda.synchronize()
    lat.perf_reset()
    # mode 2: ONE hipEvent pair on the step-kernel stream around the K timed
    # launches (per-launch dispatch events cost ~4 us of wall per step, see
    # DESIGN.md §Measurement); avg launch = region / K, inter-kernel gaps included.
    lat.set_profiling(0 if a.no_profile_events else 2)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lat.step(a.steps)
    lat.sync()
    torch.cuda.synchronize()
    barrier()
    t = time.perf_counter() - t0
    perf = lat.perf()
    lat.set_profiling(0)
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    # sanity: the field stayed finite and bounded (no guard hits)
    m = lat.moments()
    sites_local = lat.nz_local * L * L
    total_updates = float(shape[0] * shape[1] * shape[2]) * a.steps
    value = total_updates / t
    if perf["step_kernel_launches"] > 0:
        # region mean per step on the (interior) step-kernel stream; with slabs it
        # spans interior + halo + boundary, so charge all local sites to it
        avg_ms = perf["step_kernel_ms"] / perf["step_kernel_launches"]
        sites_per_launch = sites_local
    else:
        avg_ms = t * 1e3 / a.steps
        sites_per_launch = sites_local
    # two-step fused launches (phi4_tb2_kernel) update every site twice
    kname = lat.kernel_name
    spl = 2 if "2 steps per launch" in kname else 1
    launch_ms = avg_ms * spl
    achieved = BYTES_PER_SITE * sites_per_launch * spl / (launch_ms * 1e-3) / 1e9
    out = None
    if rank == 0:
        copy = None
        try:
            import ctypes
            g = ctypes.c_double()
            if _lib.load().sq_copy_bandwidth(local, 1 << 30, 20, ctypes.byref(g)) == 0:
                copy = round(g.value, 1)
        except Exception:
            copy = None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "site-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": t * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (phi0 = 0.1*Philox normal, seed 0x5EED)",
            "config": {
                "workload": f"phi^4 3-D Langevin step, {L}^3 fp32 per GPU (BASELINE configs[1]"
                            f"{'' if world == 1 else ', weak-scaled slabs = configs[3]'})" if not a.strong else
                            f"phi^4 3-D Langevin step, {L}^3 fp32 split over {world} GPU(s) (BASELINE configs[4], strong)",
                "lattice": list(shape),
                "per_gpu": [L, L, lat.nz_local],
                "dtau": a.dtau, "m2": 1.0, "lambda": 1.0,
                "ghost_depth": lat.ghost[0] if slab_path else None,
                "parallelism": "single GPU, one stream" if not slab_path else
                               f"z-slab x{world} ({a.comm if world == 1 else 'rccl'}), halo + boundary planes on "
                               f"stream B, interior on stream A",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": pmc_traffic(L, world, kname),
                "kernel": kname,
                "timing": "hipEvent pair on the kernel stream around the timed launches (region mean)"
                          if perf["step_kernel_launches"] > 0 else "wall clock",
                "steps_per_launch": spl,
                "algorithmic_bytes_per_launch": BYTES_PER_SITE * sites_per_launch * spl,
                "avg_launch_us": round(launch_ms * 1e3, 3),
                "avg_step_us": round(avg_ms * 1e3, 3),
                "launches_timed": perf["step_kernel_launches"] // spl,
                # the least HBM traffic a launch can have (one read + one write
                # of the field) and the rate it moved at
                "hbm_min_bytes_per_launch": BYTES_PER_SITE * sites_per_launch,
                "hbm_min_GBps": round(BYTES_PER_SITE * sites_per_launch / (launch_ms * 1e-3) / 1e9, 1),
            },
            "hbm_copy_peak_GBps": copy,
            "field_check": {"rms": (m["sum2"] / sites_local) ** 0.5, "maxabs": m["maxabs"]},
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(L, a.dtau, a.cpu_seconds)
        else:
            out["cpu_baseline"] = None
    lat.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
