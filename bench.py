"""bench.py -- lattice-site Langevin updates/s of the 3-D φ⁴ fp32 step on MI355X.

Workload (BASELINE.json configs[1]): a 256^3 fp32 lattice
PER GPU, periodic, Δτ = 0.01, m² = 1, λ = 1, φ₀ = 0.1·normal; one "step" = one
Langevin update of every site (sq_step).  N = 1: one GPU, one HIP stream, z
wraps in-kernel.  N > 1: one process per GPU, weak scaling, global lattice
256 x 256 x (256 N) cut into z-slabs, deep ghost zones exchanged over RCCL
(xGMI) on a second stream, overlapped with the interior planes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size L] [--strong]

With --gpus N > 1 and no torch.distributed launcher around it, the process
spawns the N rank processes itself (fresh interpreters, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, before anything touches a GPU) and relays rank 0's
line.

Timing: first a clock-settle phase (--settle-ms of steps, untimed, reported as
`settle_ms` / `settle_steps`: the short driver invocation --warmup 5 would
otherwise time ramping clocks), then W warm-up steps, then EXACTLY K timed steps
bracketed by barrier + device synchronisation; `value` = all site updates of
all ranks / max over ranks of that wall time.  `roofline.achieved` = 8
algorithmic bytes per site update x the updates of one launch
/ the mean launch duration from one hipEvent pair on the kernel's own stream
around the K timed steps (`frac_kernel`); `frac_wall` is the same bytes over
the wall time behind `value`; `frac_real` is the real HBM bytes of a launch
(the committed rocprofv3 PMC summary of this command) over the same launch time
-- the physical roofline, which the algorithmic figure (8 B per update, the
fused kernel moving the field once per two updates) cannot show.

Also in the line: `multi_rank_check` (stochquant_amd/verify.py: every rank's
slab after a fixed check protocol against the golden digests of a single-GPU
run of the same global lattice -- "pass" / "fail"), and, in the default N = 1
run, `c3_512`: BASELINE configs[2] (512^3, HBM-resident) measured the same way
in the same invocation, with its own roofline and CPU sample.  Prints ONE JSON
line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--settle-ms", type=float, default=1500.0,
                    help="untimed steps for at least this long before the warm-up (clock settle)")
    ap.add_argument("--size", type=int, default=256, help="per-GPU lattice edge (default 256 = config C2)")
    ap.add_argument("--dtau", type=float, default=0.01)
    ap.add_argument("--comm", choices=["auto", "rccl", "p2p", "loopback"], default="auto",
                    help="auto: one slab at N=1, RCCL slabs at N>1; p2p: peer-pointer halos (IPC, no RCCL) "
                         "at any N; rccl/p2p/loopback force the slab path at N=1 (self-exchange / --slabs "
                         "slabs on one GPU) to exercise it")
    ap.add_argument("--slabs", type=int, default=2)
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on GPU 0 (rehearses the multi-process --comm p2p path on a one-GPU box; "
                         "the ranks then share one device, so the rate is not a scaling figure)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (config C5): the --size^3 lattice is split over the N GPUs "
                         "instead of --size^3 per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of the CPU sample")
    ap.add_argument("--no-profile-events", action="store_true",
                    help="no hipEvents in the timed region (roofline.achieved then uses wall time)")
    ap.add_argument("--no-check", action="store_true", help="skip the multi_rank_check protocol")
    ap.add_argument("--corrupt-rank", type=int, default=-1,
                    help="(tests) flip one value of this rank's slab before its check digest")
    ap.add_argument("--no-c3", action="store_true", help="skip the 512^3 (configs[2]) sub-record of the default run")
    ap.add_argument("--cpu-seconds-c3", type=float, default=8.0, help="target wall time of the 512^3 CPU sample")
    ap.add_argument("--dry-run", action="store_true",
                    help="set up the ranks and their process group, print each rank's slab and deep-halo "
                         "schedule, touch no GPU (tests the multi-rank launch path on a CPU host)")
    return ap.parse_args()


def dry_run(a, world, rank, local, dist):
    """The multi-rank set-up without a device: every rank reports its slab, its
    device ordinal and the first block's schedule; rank 0 prints them."""
    from stochquant_amd.decomp import block_plan, slab_bounds
    L = a.size
    Lz = L if a.strong else L * world
    z0, z1 = slab_bounds(Lz, world, rank)
    g = max(1, min(16, (z1 - z0) // 16))
    info = {"rank": rank, "local_rank": local, "world": world, "slab": [z0, z1], "ghost": g,
            "plan": [o["op"] for o in block_plan(z1 - z0, g, g)] if world > 1 else None}
    allinfo = [None] * world
    if world > 1:
        dist.all_gather_object(allinfo, info)
    else:
        allinfo = [info]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": allinfo}), flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """Start n rank processes of this script (no GPU call has been made here),
    relay rank 0's stdout, return the worst exit code.  A rank that fails ends
    the others (they would otherwise wait in the rendezvous or a collective)."""
    import threading
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read().decode()), daemon=True)
    reader.start()
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    rcs = [p.wait() for p in procs]
    reader.join(timeout=10)
    sys.stdout.write("".join(out))
    sys.stdout.flush()
    return max(rcs, key=abs)


def cpu_share():
    """Host CPUs this job may use: the affinity mask, bounded by a cgroup quota."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(L, dtau, target_s):
    """Oracle (C port of the same step, OpenMP over the job's CPU share) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/baseline infrastructure only: timed as the CPU baseline, never as the product
    oracle.build()
    cores = cpu_share()
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
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{n} steps of the {L}^3 fp32 phi^4 Langevin step (oracle/orc_phi4.c, OpenMP, "
                      f"{cores} threads = this job's CPU share of {os.cpu_count()} host CPUs), {dt:.2f} s"}


def pmc_record(L, nranks, kernel):
    """The committed rocprofv3 PMC summary for this workload and kernel, if any (it is
    measured by scripts/pmc_r02.sh on this same command, not inside this run)."""
    for name in (f"pmc_traffic_{L}.json", "pmc_traffic.json"):
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("size") == L:
            break
    else:
        return None, None
    k = kernel.split("<")[0]
    if d.get("size") == L and d.get("nranks", 1) == nranks and k and k in d.get("kernel", ""):
        return d, os.path.relpath(path, ROOT)
    return None, None


def make_lattice(a, shape, world, rank, local):
    """The bench's lattice for this rank: one periodic slab at N = 1, RCCL z-slabs
    at N > 1 (or the transport --comm names)."""
    from stochquant_amd import Phi4Lattice, connect_p2p, unique_id
    import torch.distributed as dist
    kw = dict(dtau=a.dtau, m2=1.0, lam=1.0, seed=0x5EED, device=local)
    if a.comm == "p2p":
        lat = Phi4Lattice(shape, comm="p2p", nranks=world, rank=rank, **kw)
        if world > 1:
            connect_p2p(lat)
        else:
            lat.p2p_connect([lat.p2p_handle()])
    elif world > 1:
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        lat = Phi4Lattice(shape, comm="rccl", nranks=world, rank=rank, comm_id=obj[0], **kw)
    elif a.comm == "rccl":
        lat = Phi4Lattice(shape, comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
    elif a.comm == "loopback":
        lat = Phi4Lattice(shape, comm="loopback", nslabs=a.slabs, **kw)
    else:
        lat = Phi4Lattice(shape, **kw)
    return lat, (world > 1 or a.comm != "auto")


def measure(a, lat, world, slab_path):
    """Settle, warm-up, EXACTLY a.steps timed steps (barrier + device sync on both
    sides, max over ranks), then the roofline pass: the same steps again with one
    hipEvent pair on the step-kernel stream.  Returns (wall seconds, perf,
    settle_ms, settle_steps)."""
    import torch
    import torch.distributed as dist

    def barrier():
        if world > 1:
            dist.barrier()

    if slab_path:
        # setup: the timed trial blocks of the multi-rank slab path (one call long
        # enough for all of them), 3 x G steps per candidate (G, core pairs, rims)
        # in {(4,1,A), (8,1,A), (16,1,A), (16,0), (16,2|4,A|B), (16,1,A, other edge_first)}: 372 steps
        lat.step(400)
    # clock settle: untimed batches until settle_ms have passed on rank 0 (every
    # rank runs the same batches: the slab exchanges must pair up)
    settle_steps = 0
    t_settle = time.perf_counter()
    while True:
        lat.step(50)
        lat.sync()
        settle_steps += 50
        go = torch.tensor([1 if (time.perf_counter() - t_settle) * 1e3 < a.settle_ms else 0], dtype=torch.int32)
        if world > 1:
            dist.broadcast(go, src=0)
        if not int(go.item()):
            break
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    lat.step(a.warmup)
    # host bookkeeping while the warm-up steps run, so the device idles only
    # for the one synchronisation before the timed region (an idle gap lets the
    # clocks drop again).  The wall-timed region carries no instrumentation.
    lat.perf_reset()
    lat.set_profiling(0)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    lat.step(a.steps)
    torch.cuda.synchronize()   # hipDeviceSynchronize: every stream of the library's slabs
    barrier()
    t = time.perf_counter() - t0
    lat.sync()                 # the library's own join + error check, outside the timed region
    perf = lat.perf()
    if not a.no_profile_events:
        # roofline pass: the same K steps again, right behind, with ONE hipEvent
        # pair on the step-kernel stream around their launches (mode 2; avg step
        # = region / K, inter-kernel gaps included).  The pair's two marker
        # packets cost ~12 us of wall per region (0.6 us per step at K = 20,
        # profiles/r02/ab_events.log), so they stay out of the region `value`
        # is timed on; per-launch dispatch events cost ~4 us per step.
        lat.perf_reset()
        lat.set_profiling(2)
        torch.cuda.synchronize()
        barrier()
        lat.step(a.steps)
        torch.cuda.synchronize()
        barrier()
        lat.sync()
        perf = lat.perf()
        lat.set_profiling(0)
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    return t, perf, settle_ms, settle_steps


def roofline(a, lat, L, world, slab_path, t, perf, nslabs, sites_local):
    """The bench line's roofline object for the dominant (step) kernel."""
    value = float(sites_local * world) * a.steps / t if not a.strong else None
    launches = max(1, perf["kernel_launches"])
    spl = perf["steps"] * nslabs / launches          # steps per launch, measured (2 = two-step fused)
    if perf["step_kernel_launches"] > 0:
        # event region on the (interior) step-kernel stream: it spans every
        # launch of the timed steps, so charge all local sites to it
        step_ms = perf["step_kernel_ms"] / perf["step_kernel_launches"]
    else:
        step_ms = t * 1e3 / a.steps
    launch_ms = step_ms * spl
    achieved = BYTES_PER_SITE * sites_local / (step_ms * 1e-3) / 1e9
    kname = lat.kernel_name
    rec, rec_path = pmc_record(L, world, kname) if not slab_path else (None, None)
    fused = "tb2" in kname and perf.get("fused_steps", 0) >= 0.5 * perf["steps"]
    r = {
        # the fused kernel moves the field once per two updates
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4),
        "frac_kernel": round(achieved / HBM_PEAK_GBPS, 4),
        "achieved_is": "algorithmic bytes (8 B per site update, SURVEY.md §8d) / time",
        "traffic": rec.get("hbm_bytes_per_launch") if rec else None,
        "traffic_source": (f"cached: {rec_path}, rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes of this "
                           f"bench command (not measured inside this run)") if rec else None,
        "kernel": kname,
        "timing": "hipEvent pair on the kernel stream around a second pass of the same K steps right "
                  "after the wall-timed region (region mean)"
                  if perf["step_kernel_launches"] > 0 else "wall clock",
        "steps_per_launch": round(spl, 3),
        "kernel_launches_timed": perf["kernel_launches"],
        "algorithmic_bytes_per_launch": round(BYTES_PER_SITE * sites_local * spl),
        "avg_launch_us": round(launch_ms * 1e3, 3),
        "avg_step_us": round(step_ms * 1e3, 3),
        # the least HBM traffic a launch can have (one read + one write
        # of the field) and the rate it moved at
        "hbm_min_bytes_per_launch": BYTES_PER_SITE * sites_local,
        "hbm_min_GBps": round(BYTES_PER_SITE * sites_local / (launch_ms * 1e-3) / 1e9, 1),
    }
    if rec:
        # headroom the algorithmic figure cannot show (it counts 8 B per update,
        # the fused kernel moves the field once per two): the real HBM bytes of
        # a launch (PMC) over this run's launch time, the per-SIMD VALU issue
        # utilisation and the launch busy fraction of the committed counters
        tb = rec.get("hbm_bytes_per_launch")
        if tb:
            r["real_GBps"] = round(tb / (launch_ms * 1e-3) / 1e9, 1)
            r["frac_real"] = round(tb / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        for k in ("valu_util_simd", "valu_issue_util_simd", "avg_resident_waves_per_simd", "valu_util_method",
                  "pmc_kernel_us"):
            if rec.get(k) is not None:
                r[k] = rec[k]
    if fused and not slab_path and world == 1:
        r.update(busy_fraction(lat))
    return r, value, fused


def busy_fraction(lat, reps=5):
    """Launch busy fraction from per-block clock stamps of a few fused launches
    (sq_phi4_block_stamps, measured in this run): the blocks' summed durations
    over blocks x launch span (first start to last end), median of `reps`
    launches; with the block-end percentiles (us from the launch's first start)."""
    import numpy as np
    fr, spans, ends = [], [], []
    for _ in range(reps):
        st, en = lat.block_stamps()
        t0 = st.min()
        span = float(en.max() - t0)
        fr.append(float((en - st).sum()) / (len(st) * span))
        spans.append(span * 1e-2)          # 100 MHz ticks -> us
        ends.append(np.percentile((en - t0) * 1e-2, [10, 50, 90]))
    i = int(np.argsort(fr)[len(fr) // 2])
    return {"busy_fraction": round(fr[i], 3), "busy_launch_span_us": round(spans[i], 2),
            "busy_block_end_us_p10_p50_p90": [round(float(x), 2) for x in ends[i]],
            "busy_source": "sq_phi4_block_stamps: per-block s_memrealtime start/end of the fused launch, "
                           f"median of {reps} launches in this run"}


def cpu_baseline_c3(L, dtau, target_s):
    try:
        return cpu_baseline(L, dtau, target_s)
    except Exception as e:  # the GPU record stands without it
        return {"error": str(e)[:200]}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    a.gpus = world
    import torch
    import torch.distributed as dist
    from stochquant_amd import _lib, verify
    _lib.load()  # fail loudly if the HIP library is missing
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one node by contract: RCCL's bootstrap over loopback (data moves over xGMI)
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if a.dry_run:
        dry_run(a, world, rank, local, dist)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    L = a.size
    shape = (L, L, L) if a.strong else (L, L, L * world)
    lat, slab_path = make_lattice(a, shape, world, rank, local)
    lat.init_field(0.1)
    t, perf, settle_ms, settle_steps = measure(a, lat, world, slab_path)
    # sanity: the field stayed finite and bounded (no guard hits)
    m = lat.moments()
    sites_local = lat.nz_local * L * L
    total_updates = float(shape[0] * shape[1] * shape[2]) * a.steps
    value = total_updates / t
    nslabs = a.slabs if (world == 1 and a.comm == "loopback") else 1
    rl, _, fused = roofline(a, lat, L, world, slab_path, t, perf, nslabs, sites_local)
    achieved_wall = BYTES_PER_SITE * value / 1e9
    rl["frac_wall"] = round(achieved_wall / HBM_PEAK_GBPS, 4)
    rl["achieved_wall"] = round(achieved_wall, 1)
    # self-check (verify.py): the check protocol's slab digests against the
    # golden ones of a single-GPU run of the same global lattice, every rank
    check = "skipped"
    if not a.no_check and a.dtau == verify.CHECK_PARAMS["dtau"]:
        d = verify.run_protocol(lat, corrupt=(rank == a.corrupt_rank))
        digests = [None] * world
        if world > 1:
            dist.all_gather_object(digests, d)
        else:
            digests = [d]
        check = verify.check(digests, shape, world)
    ghost = lat.ghost[0] if slab_path else None
    schedule = lat.schedule if slab_path else None
    kname = lat.kernel_name
    nz_local = lat.nz_local
    lat.close()
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
        cfg_idx = {256: 1, 512: 2}.get(L)
        if a.strong:
            workload = f"phi^4 3-D Langevin step, {L}^3 fp32 split over {world} GPU(s) (BASELINE configs[4], strong)"
        elif world > 1:
            workload = f"phi^4 3-D Langevin step, {L}^3 fp32 per GPU, weak-scaled z-slabs (BASELINE configs[3])"
        else:
            workload = (f"phi^4 3-D Langevin step, {L}^3 fp32 on one GPU"
                        + (f" (BASELINE configs[{cfg_idx}])" if cfg_idx is not None else ""))
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "site-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "settle_ms": round(settle_ms, 1),
            "settle_steps": settle_steps,
            "ms_per_step": t * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (phi0 = 0.1*Philox normal, seed 0x5EED)",
            "config": {
                "workload": workload,
                "lattice": list(shape),
                "per_gpu": [L, L, nz_local],
                "dtau": a.dtau, "m2": 1.0, "lambda": 1.0,
                "ghost_depth": ghost,
                "block_schedule": schedule,
                "parallelism": "single GPU, one stream" if not slab_path else
                               f"z-slab x{world} ({a.comm if world == 1 or a.comm == 'p2p' else 'rccl'}), halo exchange on "
                               f"stream B, interior on stream A",
            },
            "roofline": rl,
            "multi_rank_check": check,
            "multi_rank_check_protocol": (f"init 0.1*normal, step counter 0, {verify.CHECK_STEPS} steps; every "
                                          f"rank's slab digest vs the golden single-GPU run "
                                          f"(stochquant_amd/golden_slabs.json)"),
            "hbm_copy_peak_GBps": copy,
            "field_check": {"rms": (m["sum2"] / sites_local) ** 0.5, "maxabs": m["maxabs"]},
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(L, a.dtau, a.cpu_seconds)
        else:
            out["cpu_baseline"] = None
    # config C3 (BASELINE configs[2], 512^3 on one GPU) in the same invocation:
    # the same settle, warm-up and --steps, its own roofline and CPU sample
    if world == 1 and not a.strong and a.comm == "auto" and L == 256 and not a.no_c3:
        L3 = 512
        lat3, _ = make_lattice(a, (L3, L3, L3), 1, 0, local)
        lat3.init_field(0.1)
        t3, perf3, settle3, ssteps3 = measure(a, lat3, 1, False)
        sites3 = L3 ** 3
        rl3, value3, _ = roofline(a, lat3, L3, 1, False, t3, perf3, 1, sites3)
        rl3["frac_wall"] = round(BYTES_PER_SITE * value3 / 1e9 / HBM_PEAK_GBPS, 4)
        m3 = lat3.moments()
        lat3.close()
        out["c3_512"] = {
            "config": {"workload": "phi^4 3-D Langevin step, 512^3 fp32 on one GPU (BASELINE configs[2], "
                                   "HBM-resident: 2 x 512 MiB > the 256 MiB Infinity Cache)",
                       "lattice": [L3, L3, L3], "dtau": a.dtau, "m2": 1.0, "lambda": 1.0},
            "value": value3, "unit": "site-updates/s", "steps": a.steps, "warmup": a.warmup,
            "settle_ms": round(settle3, 1), "settle_steps": ssteps3, "ms_per_step": t3 * 1e3 / a.steps,
            "roofline": rl3,
            "field_check": {"rms": (m3["sum2"] / sites3) ** 0.5, "maxabs": m3["maxabs"]},
            "cpu_baseline": None if a.no_cpu_baseline else cpu_baseline_c3(L3, a.dtau, a.cpu_seconds_c3),
        }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
