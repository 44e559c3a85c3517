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
all ranks / max over ranks of that wall time.

Roofline: the dominant kernel is the two-step fused kernel,
which moves the field once per two updates and is bound by VALU issue, not
HBM.  `bound` "valu", `frac` = the launch's VALU-busy SIMD cycles (4 x
SQ_ACTIVE_INST_VALU from the committed rocprofv3 PMC record of this same
command, profiles/r06/driver_profile.json) / (1024 SIMDs x 2.4 GHz x the launch
time measured here with dispatch events, as rocprofv3's kernel trace measures
it).  Beside it: `frac_algorithmic` (8 B per site update, SURVEY.md §8d, over
the same time -- saturates by construction under two-step temporal blocking),
`frac_hbm_real` (the PMC bytes of a launch over that time) and
`frac_algorithmic_wall` (8 B per update over the wall time behind `value`).

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
    ap.add_argument("--no-c1", action="store_true", help="skip the 32,768-site QM1D chain (configs[0]) sub-record")
    ap.add_argument("--c1-frames", type=int, default=8, help="timed 1000-step frames of the C1 chain")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the 1024^3 strong-scaling (configs[4]) sub-record, run at every N")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the frames_256 / slab_1gpu / c1_phi4_32 sub-records of the default run")
    ap.add_argument("--cpu-loops-c1", type=int, default=1000,
                    help="steps of the C1 CPU sample (the reference's serial semantics on one core)")
    ap.add_argument("--rank-timeout", type=float, default=None,
                    help="deadline (s) for the whole run of every rank; on expiry rank 0 prints one JSON line with "
                         "'error' and every rank's last phase and the ranks exit 3 (default: 300 s + 2 ms per "
                         "step; 0 = none)")
    ap.add_argument("--inject-stall", default=None,
                    help="(tests) RANK:SECONDS -- this rank sleeps that long in its phase 'stall' after the "
                         "rendezvous")
    ap.add_argument("--inject-error", type=int, default=None,
                    help="(tests) this rank raises after the rendezvous")
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


def rank_deadline(a):
    """Seconds every rank of the run may take in all (--rank-timeout, 0 = none)."""
    if a.rank_timeout is not None:
        return a.rank_timeout
    return 300.0 + 2e-3 * (a.steps + a.warmup)


def spawn_ranks(n, deadline_s):
    """Start n rank processes of this script (no GPU call has been made here),
    relay rank 0's stdout, return the worst exit code.  A rank that fails ends
    the others (they would otherwise wait in the rendezvous or a collective).
    The ranks run their own deadline (stochquant_amd.rankwatch); 30 s after it
    this parent kills them and prints the error line itself with every rank's
    last reported phase."""
    import threading
    from stochquant_amd import rankwatch
    port = str(_free_port())
    pdir = rankwatch.phase_dir(port)
    os.makedirs(pdir, exist_ok=True)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, SQ_PHASE_DIR=pdir)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read().decode()), daemon=True)
    reader.start()
    t_end = time.time() + deadline_s + 30.0 if deadline_s > 0 else None
    expired = False
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            break
        if t_end is not None and time.time() > t_end:
            expired = True
            break
        time.sleep(0.2)
    phases = rankwatch.read_phases(pdir, n)
    # SIGTERM first: rank 0 then prints the line with every rank's phase
    # (a failed rank's phase holds its error); SIGKILL what is left after 5 s
    for p in procs:
        if p.poll() is None:
            p.terminate()
    t_kill = time.time() + 5.0
    while any(p.poll() is None for p in procs) and time.time() < t_kill:
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.kill()
    rcs = [p.wait() for p in procs]
    reader.join(timeout=10)
    text = "".join(out)
    if expired and not any(l.startswith("{") for l in text.splitlines()):
        text += rankwatch.error_line(METRIC, n, deadline_s, phases,
                                     f"ranks did not finish within the deadline of {deadline_s:.0f} s + 30 s; "
                                     f"killed by the spawning process") + "\n"
    sys.stdout.write(text)
    sys.stdout.flush()
    if expired:
        return rankwatch.EXIT_DEADLINE
    # rank 0's own status first (its deadline exit is 3); the others were
    # killed after it ended; a signal becomes 128 + signo
    worst = rcs[0] if rcs[0] != 0 else max(rcs, key=abs)
    return worst if worst >= 0 else 128 - worst


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


PROFILE = os.path.join("profiles", "r06", "driver_profile.json")
PROFILE_TIMING_TOL = 0.03       # the record's rocprof launch time must be within 3 % of this run's
N_SIMD = 1024                   # 256 CUs x 4 SIMDs
CLOCK_MHZ = 2400.0              # peak engine clock (MI355X_MICROARCH.md)
VALU_PEAK = N_SIMD * CLOCK_MHZ / 1e3   # G SIMD-cycles/s: every SIMD issuing VALU every cycle


def short_kernel(name):
    """'void sq::(anonymous namespace)::phi4_tb2_kernel<...>(sq::Phi4StepArgs)' -> 'phi4_tb2_kernel<...>'."""
    name = name.split("(sq::")[0] if "(sq::" in name else name
    return name.split("::")[-1].strip()


def pmc_record(L, launched, build, path=None):
    """The committed rocprofv3 record of the driver's invocation for this lattice
    (profiles/r06/driver_profile.json, made by scripts/r06/driver_prof.sh +
    scripts/driver_profile.py from `python3 bench.py --steps 20 --warmup 5`,
    not measured inside this run): PMC HBM bytes and VALU-busy cycles per launch
    of the fused kernel, and its rocprof dispatch durations.

    The record is used only for the binary and launch it describes: its
    phi4 build id (the hash of the φ⁴ kernels' code object, sq_build_id) must be
    the loaded library's, its kernel the template instance this run launched
    most (sq_phi4_launch_info), its grid the same.  Returns (record, path,
    None), or (None, path, reason) when there is a record for this lattice
    that does not describe this run (a stale profile), or (None, None, None)
    when there is none."""
    rel = path or PROFILE
    try:
        with open(os.path.join(ROOT, rel)) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None, None
    rec = d.get("configs", {}).get(str(L))
    if not rec:
        return None, None, None
    why = []
    if rec.get("build_id_phi4") != build.get("phi4"):
        why.append(f"build id {rec.get('build_id_phi4')} != loaded {build.get('phi4')}")
    if short_kernel(rec.get("kernel", "")) != launched.get("kernel"):
        why.append(f"kernel {short_kernel(rec.get('kernel', ''))} != launched {launched.get('kernel')}")
    if rec.get("grid") != launched.get("grid"):
        why.append(f"grid {rec.get('grid')} != launched {launched.get('grid')}")
    if why:
        return None, rel, "; ".join(why)
    return rec, rel, None


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

        def rccl():
            q = Phi4Lattice(shape, comm="rccl", nranks=world, rank=rank, comm_id=obj[0], **kw)
            try:  # one deep-halo block: the first cross-device exchanges, before anything is timed
                q.step(16)
                q.sync()
            except Exception:
                q.close()
                raise
            return q

        def p2p():
            q = Phi4Lattice(shape, comm="p2p", nranks=world, rank=rank, **kw)
            connect_p2p(q)
            return q

        # RCCL with nranks > 1 first runs on the driver's node: should its bring-up
        # fail on any rank (an error, bounded by the nonblocking init's timeout),
        # every rank moves to the copy-engine P2P transport together
        lat, why = open_with_fallback(rccl, p2p, world, dist)
        a.transport = "rccl" if why is None else "p2p"
        a.transport_fallback = why
    elif a.comm == "rccl":
        lat = Phi4Lattice(shape, comm="rccl", nranks=1, rank=0, comm_id=unique_id(), **kw)
    elif a.comm == "loopback":
        lat = Phi4Lattice(shape, comm="loopback", nslabs=a.slabs, **kw)
    else:
        lat = Phi4Lattice(shape, **kw)
    return lat, (world > 1 or a.comm != "auto")


def open_with_fallback(make_primary, make_fallback, world, dist):
    """Every rank opens the primary transport; if it failed on ANY rank (agreed
    by a MIN all-reduce over the host group), every rank closes what it opened
    and opens the fallback instead.  Returns (lattice, None) or (lattice,
    reason) -- the reason is this rank's error, or that another rank failed."""
    import torch
    lat, err = None, None
    try:
        lat = make_primary()
    except Exception as e:   # the library's error (SQ_E_COMM / SQ_E_HIP), not a hang
        err = e
    ok = torch.tensor([0 if lat is None else 1], dtype=torch.int32)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 1:
        return lat, None
    if lat is not None:
        lat.close()
    why = f"{type(err).__name__}: {err}" if err is not None else "the primary transport failed on another rank"
    return make_fallback(), why


def measure(a, lat, world, slab_path, watch=None):
    """Settle, warm-up, EXACTLY a.steps timed steps (barrier + device sync on both
    sides, max over ranks), then the roofline pass: the same steps again with one
    hipEvent pair on the step-kernel stream.  Returns (wall seconds, perf,
    settle_ms, settle_steps)."""
    import torch
    import torch.distributed as dist

    def barrier():
        if world > 1:
            dist.barrier()

    def phase(name):
        if watch is not None:
            watch.phase(name)

    if slab_path:
        phase("trial_blocks")
        # setup: the timed trial blocks of the multi-rank slab path (one call long
        # enough for all of them), 3 x G steps per candidate (G, core pairs, rims)
        # in {(4,1,A), (8,1,A), (16,1,A), (16,0), (16,2|4,A|B), (16,1,A, other edge_first),
        # (16, exchange in order on A)}: 420 steps
        lat.step(440)
    # clock settle: untimed batches until settle_ms have passed on rank 0 (every
    # rank runs the same batches: the slab exchanges must pair up)
    phase("settle")
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
    phase("warmup")
    lat.step(a.warmup)
    # host bookkeeping while the warm-up steps run, so the device idles only
    # for the one synchronisation before the timed region (an idle gap lets the
    # clocks drop again).  The wall-timed region carries no instrumentation.
    lat.perf_reset()
    lat.set_profiling(0)
    torch.cuda.synchronize()
    barrier()
    phase("timed")
    t0 = time.perf_counter()
    lat.step(a.steps)
    torch.cuda.synchronize()   # hipDeviceSynchronize: every stream of the library's slabs
    barrier()
    t = time.perf_counter() - t0
    lat.sync()                 # the library's own join + error check, outside the timed region
    perf = lat.perf()
    if not a.no_profile_events:
        phase("roofline_pass")
        # roofline pass: the same K steps again, right behind the wall-timed
        # region (whose launches carry no instrumentation), with ONE hipEvent
        # pair on the step-kernel stream around their launches (mode 2; avg
        # launch = region / launches, inter-kernel gaps included).  In one
        # profiled run this mean agreed with rocprofv3's average dispatch
        # duration of the same kernel within 0.6 % (32.16 vs 32.35 us), while
        # per-launch dispatch events (mode 1) read 35.3 us: they perturb the
        # launches they time (profiles/r04/README.md).
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
    """The bench line's roofline object for the dominant (step) kernel.

    The fused two-step kernel is bound by VALU issue, not HBM:
    it moves the field once per two updates, so 8 algorithmic bytes per update
    over its time can exceed the HBM peak by construction.  For it `bound` is
    "valu" and `frac` the physical fraction: the launch's VALU-busy SIMD cycles
    (4 x SQ_ACTIVE_INST_VALU from the committed PMC record of this very
    command) over 1024 SIMDs x 2.4 GHz x the launch time measured here.
    `frac_algorithmic` keeps the contract's 8 B/update figure, `frac_hbm_real`
    the PMC bytes of a launch over the same time."""
    value = float(sites_local * world) * a.steps / t if not a.strong else None
    launches = max(1, perf["kernel_launches"])
    spl = perf["steps"] * nslabs / launches          # steps per launch, measured (2 = two-step fused)
    kname = lat.kernel_name
    fused = "tb2" in kname and perf.get("fused_steps", 0) >= 0.5 * perf["steps"]
    if perf["step_kernel_launches"] > 0:
        # one event pair on the (interior) step-kernel stream around the K steps:
        # it spans every launch of them, so charge all local sites to it
        step_ms = perf["step_kernel_ms"] / perf["step_kernel_launches"]
        timing = ("hipEvent pair on the kernel stream around a second pass of the same K steps right after the "
                  "wall-timed region (region mean, inter-kernel gaps included)")
    else:
        step_ms = t * 1e3 / a.steps
        timing = "wall clock"
    launch_ms = step_ms * spl
    alg = BYTES_PER_SITE * sites_local / (step_ms * 1e-3) / 1e9      # GB/s, 8 B per site update
    launched = lat.launch_info()        # the kernel the roofline pass launched most, and its grid
    from stochquant_amd import _lib
    build = _lib.build_id()
    rec, rec_path, stale = pmc_record(L, launched, build) if (not slab_path and world == 1) else (None, None, None)
    r = {"kernel": launched["kernel"] or kname, "grid_threads": launched["grid"], "kernel_config": kname,
         "build_id": build, "timing": timing, "steps_per_launch": round(spl, 3),
         "kernel_launches_timed": perf["kernel_launches"],
         "avg_launch_us": round(launch_ms * 1e3, 3), "avg_step_us": round(step_ms * 1e3, 3)}
    valu = None
    if fused and rec and rec.get("valu_busy_cycles_per_launch"):
        valu = rec["valu_busy_cycles_per_launch"] / (launch_ms * 1e-3) / 1e9    # G SIMD-cycles/s
    if fused and valu is not None:
        r.update({
            "bound": "valu",
            "achieved": round(valu, 1),
            "peak": VALU_PEAK,
            "unit": "G VALU-busy SIMD-cycles/s",
            "frac": round(valu / VALU_PEAK, 4),
            "achieved_is": ("VALU-issue cycles of one launch (4 x SQ_ACTIVE_INST_VALU, committed PMC record of "
                            "this command, same build id / kernel / grid) / the launch time measured here; "
                            "peak = 1024 SIMDs x 2.4 GHz"),
        })
    elif fused and stale:
        # a record exists for this lattice but describes another binary or launch:
        # no number rather than a confident wrong one
        r.update({"bound": "valu", "achieved": None, "peak": VALU_PEAK, "unit": "G VALU-busy SIMD-cycles/s",
                  "frac": None, "stale_profile": True, "stale_reason": stale,
                  "achieved_is": f"not computed: {rec_path} does not describe this run ({stale})"})
    elif fused:
        # no PMC record (other lattice sizes, slab paths, N > 1): the contract's
        # algorithmic bytes, labelled as such -- a fused launch moves the field
        # once per two updates, so this ratio is not an HBM measurement
        r.update({
            "bound": "hbm_algorithmic",
            "achieved": round(alg, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(alg / HBM_PEAK_GBPS, 4),
            "achieved_is": ("algorithmic bytes (8 B per site update, SURVEY.md §8d) / the measured step time; no "
                            "PMC record for this run, and two-step fused launches move the field once per two "
                            "updates, so the ratio can exceed 1 and is not a measured HBM fraction"),
        })
    else:
        r.update({
            "bound": "hbm",
            "achieved": round(alg, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(alg / HBM_PEAK_GBPS, 4),
            "achieved_is": "algorithmic bytes (8 B per site update, SURVEY.md §8d) / time (one step per launch)",
        })
    r["frac_algorithmic"] = round(alg / HBM_PEAK_GBPS, 4)
    r["achieved_algorithmic_GBps"] = round(alg, 1)
    r["algorithmic_bytes_per_launch"] = round(BYTES_PER_SITE * sites_local * spl)
    r["hbm_min_bytes_per_launch"] = BYTES_PER_SITE * sites_local
    r["traffic"] = rec.get("hbm_bytes_per_launch") if rec else None
    if rec:
        r["traffic_source"] = (f"{rec_path}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) / WRITE_SIZE passes of "
                               f"`{json.load(open(os.path.join(ROOT, rec_path)))['command']}`, median per launch")
        tb = rec.get("hbm_bytes_per_launch")
        if tb:
            r["achieved_hbm_real_GBps"] = round(tb / (launch_ms * 1e-3) / 1e9, 1)
            r["frac_hbm_real"] = round(tb / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
            r["traffic_over_hbm_min"] = round(tb / (BYTES_PER_SITE * sites_local), 4)
        # the record's counts (VALU cycles, bytes) are clock-independent and
        # divided by the live launch time above; its rocprof durations describe
        # this run only when they agree with the live launch (within
        # PROFILE_TIMING_TOL) -- otherwise they are flagged and not quoted
        ratio = launch_ms * 1e3 / rec["rocprof_avg_us"] if rec.get("rocprof_avg_us") else None
        mismatch = ratio is not None and abs(ratio - 1.0) > PROFILE_TIMING_TOL
        keys = ["valu_busy_cycles_per_launch", "valu_insts_per_wave", "avg_resident_waves_per_simd"]
        if not mismatch:
            keys += ["rocprof_avg_us", "rocprof_median_us", "valu_util_simd_at_rocprof_avg"]
        for k in keys:
            if rec.get(k) is not None:
                r["profile_" + k] = rec[k]
        if ratio is not None:
            r["launch_us_vs_rocprof_avg"] = round(ratio, 4)
            r["profile_timing_mismatch"] = mismatch
    if fused and not slab_path and world == 1:
        r.update(busy_fraction(lat, step_ms))
        mhz = r.get("clock_MHz_measured")
        if mhz and r.get("frac") is not None and r.get("unit", "").startswith("G VALU"):
            # the same VALU cycles against the clock the chip actually ran at
            r["frac_at_measured_clock"] = round(r["frac"] * CLOCK_MHZ / mhz, 4)
    return r, value, fused


def busy_fraction(lat, step_ms, reps=5):
    """Launch busy fraction from per-block clock stamps of a few fused launches
    (sq_phi4_block_stamps, measured in this run): the blocks' summed durations
    over blocks x launch span (first start to last end), median of `reps`
    launches; with the block-end percentiles (us from the launch's first start).
    Each stamped launch runs behind ~5 ms of queued steps, so the chip's power
    management is in its sustained state; the blocks' shader-clock counters
    (sq_phi4_block_clocks) over their 100 MHz stamps give the clock it ran at."""
    import numpy as np
    pre = max(2, 2 * int(2.5 / step_ms))
    fr, spans, ends, mhz = [], [], [], []
    for _ in range(reps):
        lat.step(pre)
        st, en = lat.block_stamps()
        cs, ce = lat.block_clocks()
        t0 = st.min()
        span = float(en.max() - t0)
        fr.append(float((en - st).sum()) / (len(st) * span))
        spans.append(span * 1e-2)          # 100 MHz ticks -> us
        ends.append(np.percentile((en - t0) * 1e-2, [10, 50, 90]))
        ok = en > st
        mhz.append(float(np.median((ce[ok] - cs[ok]) / (en[ok] - st[ok]))) * 100.0)
    i = int(np.argsort(fr)[len(fr) // 2])
    clk = float(np.median(mhz))
    out = {"busy_fraction": round(fr[i], 3), "busy_launch_span_us": round(spans[i], 2),
           "busy_block_end_us_p10_p50_p90": [round(float(x), 2) for x in ends[i]],
           "busy_source": "sq_phi4_block_stamps: per-block s_memrealtime start/end of the fused launch, "
                          f"median of {reps} launches in this run, each behind {pre} queued steps"}
    # a plausible shader clock only (the counter's rate is the chip's, not the constant clock's)
    out["clock_MHz_measured"] = round(clk, 1) if 100.0 <= clk <= 3000.0 else None
    out["clock_source"] = ("per-block s_memtime (shader clock) over s_memrealtime (100 MHz) deltas of the stamped "
                           "launches, median; the chip holds its 1400 W package power cap by lowering the clock "
                           "(DESIGN.md §6)")
    return out


def cpu_baseline_c3(L, dtau, target_s):
    try:
        return cpu_baseline(L, dtau, target_s)
    except Exception as e:  # the GPU record stands without it
        return {"error": str(e)[:200]}


C1 = dict(N=32768, deltat=1.0, dtau=0.01, pot=0, C=1.0, loops=1000, seed=1)


def c1_cpu_baseline(loops):
    """The reference's own semantics for config C1 on one host core: the serial
    restatement of one clEnqueueNDRangeKernel of time_dev (tau_kernel.cl:25-175,
    oracle/orc_qm1d.c orc_serial_launch, shared LCG, in-order items) driven as
    tauhost.c:479-560 (oracle.SerialChain), one frame of `loops` steps."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/baseline infrastructure only: timed as the CPU baseline, never as the product
    oracle.build()
    N = C1["N"]
    f0 = (2 * C1["dtau"]) ** 0.5 * np.random.default_rng(C1["seed"]).standard_normal(N)
    ch = oracle.SerialChain(N, C1["deltat"], C1["dtau"], C1["pot"], C1["C"], loops, 12345, f0,
                            omega=C1["deltat"] * (N // 2))
    t0 = time.perf_counter()
    ch.frame()
    dt = time.perf_counter() - t0
    return {"value": N * loops / dt, "unit": "site-updates/s", "cores": 1, "kind": "port",
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"one {loops}-step frame of the {N}-site chain under the reference's serial semantics "
                      f"(oracle/orc_qm1d.c orc_serial_launch + tauhost.c's frame loop, oracle.SerialChain; "
                      f"single-threaded, as the reference's one work-group), {dt:.2f} s"}


def c1_record(a, local):
    """BASELINE configs[0] / SURVEY.md §8d C1: the 32,768-site QM1D chain, 1000-step
    Jacobi frames through the library (qm1d_frame_grid: the whole chip, one grid
    barrier per step), f0 ~ N(0, 2 dtau), potID 0, C = 1.  Site-updates/s over
    --c1-frames back-to-back frames (wall, one sync), the kernel time per frame
    from dispatch events, and the CPU baseline of the reference's semantics."""
    import numpy as np
    import torch
    from stochquant_amd import Qm1dChain
    N, loops = C1["N"], C1["loops"]
    f0 = (2 * C1["dtau"]) ** 0.5 * np.random.default_rng(C1["seed"]).standard_normal(N)
    with Qm1dChain(N, C1["deltat"], C1["dtau"], pot=C1["pot"], C=C1["C"], loops=loops, seed=C1["seed"],
                   device=local) as q:
        q.upload(f0, omega=C1["deltat"] * (N // 2))
        for _ in range(2):                   # warm-up: allocations, code objects, clocks
            q.run_frame()
        q.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        stable = [q.run_frame() for _ in range(a.c1_frames)]
        q.sync()
        t = time.perf_counter() - t0
        q.perf_reset()
        q.set_profiling(1)
        for _ in range(a.c1_frames):
            q.run_frame()
        q.sync()
        perf = q.perf()
        q.set_profiling(0)
        d = q.download()
    kern_ms = perf["step_kernel_ms"] / max(1, a.c1_frames)
    value = N * loops * a.c1_frames / t
    alg = 48.0 * N * loops / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None
    return {
        "config": {"workload": "QM1D chain, N = 32,768 sites (BASELINE configs[0] as SURVEY.md §8d C1), fp64, "
                               "Jacobi order + Philox noise, one frame = 1000 Langevin steps",
                   "N": N, "deltat": C1["deltat"], "dtau": C1["dtau"], "potID": C1["pot"], "C": C1["C"],
                   "loops": loops, "f0": "sqrt(2 dtau) * normal (seed 1)"},
        "value": value, "unit": "site-updates/s", "frames": a.c1_frames, "stable_frames": int(sum(stable)),
        "ms_per_frame": t * 1e3 / a.c1_frames,
        "kernel_ms_per_frame": round(kern_ms, 4),
        "roofline": {"bound": "latency", "achieved": round(alg, 1) if alg else None, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(alg / HBM_PEAK_GBPS, 5) if alg else None,
                     "achieved_is": "48 algorithmic B per site-step (f, x, xx0 read + written, fp64; SURVEY.md "
                                    "§8d C1) / the frame kernels' dispatch-event time; the chain is bound by one "
                                    "grid barrier + the fp64 divisions per step, not by memory (DESIGN.md §4)"},
        "field_check": {"rms": float(np.sqrt(np.mean(d["f"] ** 2)))},
        "cpu_baseline": None if a.no_cpu_baseline else c1_cpu_baseline(a.cpu_loops_c1),
    }


def frames_record(a, local, nframes=200, loops=20, rounds=8):
    """tauhost.c:479-560's unit on the north-star lattice: 20-step 256^3 frames
    (guard, stability rule, rollback, Δτ controller) decided on the device
    (sq_run_frames), against raw 20-step blocks (sq_step) in the same context
    and run: `rounds` alternating rounds of a batch of nframes / rounds frames
    and as many raw steps, in alternating order, summed per kind (one batch of
    frames timed before one block of raw steps put 1-4 points of clock-state
    difference into the overhead, round 6, scripts/r06/frames_diag.py)."""
    import numpy as np
    import torch
    from stochquant_amd import Phi4Lattice
    per = nframes // rounds
    with Phi4Lattice((256, 256, 256), dtau=a.dtau, m2=1.0, lam=1.0, seed=0x5EED, device=local, loops=loops) as L:
        L.init_field(0.1)
        L.run_frames(20)                   # warm-up: code objects, the controller, clocks
        L.step(200)
        L.sync()
        tf = tr = 0.0
        sts, dts = [], []

        def frames():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st, dt = L.run_frames(per)
            L.sync()
            sts.append(st)
            dts.append(dt)
            return time.perf_counter() - t0

        def raw():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L.step(per * loops)
            L.sync()
            return time.perf_counter() - t0

        for r in range(rounds):  # the order alternates too: whichever runs first after a sync reads differently
            if r % 2 == 0:
                tf += frames()
                tr += raw()
            else:
                tr += raw()
                tf += frames()
        m = L.moments()
    nf = per * rounds
    st, dts = np.concatenate(sts), np.concatenate(dts)
    us_f = tf * 1e6 / nf
    us_raw = tr * 1e6 / (nf * loops) * loops
    return {"config": {"workload": "phi^4 256^3 fp32, frames of 20 Langevin steps through sq_run_frames (the "
                                   "frame loop of tauhost.c:479-560 on the device: guard flag, stability rule, "
                                   "rollback, Δτ controller)", "loops": loops, "frames": nf, "rounds": rounds,
                       "method": "alternating rounds (and order) of a frame batch and as many raw steps, summed per kind",
                       "dtau0": a.dtau, "m2": 1.0, "lambda": 1.0},
            "us_per_frame": round(us_f, 2), "raw_us_per_20_steps": round(us_raw, 2),
            "overhead": round(us_f / us_raw - 1.0, 4), "stable_frames": int(st.sum()),
            "dtau_final": float(dts[-1]) if len(dts) else None,
            "value": 256 ** 3 * loops * nf / tf, "unit": "site-updates/s (frames)",
            "field_check": {"maxabs": m["maxabs"]}}


def slab_record(a, local, steps=1000, rounds=5):
    """SURVEY §8e's slab path on one GPU: the 256^3 lattice as one z-slab whose
    halo exchange goes through the product's transports to itself (RCCL
    self-exchange; P2P peer pointers), G = 16 deep halos, fused pairs, one
    rank's default schedule (the exchange in order on the interior stream
    between blocks, P2P's last pair writing its staging slot; DESIGN.md §8.3,
    reported as each context's "schedule") -- per-step time against the single periodic slab in
    the same run (the ratio is what the exchange machinery costs before any
    xGMI).  All three contexts stay open and are timed in turn, `rounds` times
    `steps` steps each after 2000 warm-up steps, medians: one measurement per
    context right after its creation read the single slab 2-5 % slow or fast
    with the clock state (round 6, scripts/r06/slab_ab.py)."""
    import statistics
    import torch
    from stochquant_amd import Phi4Lattice, unique_id
    kw = dict(dtau=a.dtau, m2=1.0, lam=1.0, seed=0x5EED, device=local)
    out, ctxs = {}, {}

    def p2p():
        L = Phi4Lattice((256, 256, 256), comm="p2p", nranks=1, rank=0, **kw)
        try:
            L.p2p_connect([L.p2p_handle()])
        except Exception:
            L.close()
            raise
        return L

    try:
        for name, mk in (("single", lambda: Phi4Lattice((256, 256, 256), **kw)),
                         ("rccl", lambda: Phi4Lattice((256, 256, 256), comm="rccl", nranks=1, rank=0,
                                                      comm_id=unique_id(), **kw)),
                         ("p2p", p2p)):
            try:
                L = mk()
                L.init_field(0.1)
                L.step(2000)
                L.sync()
                ctxs[name] = L
            except Exception as e:   # the headline record stands without it
                out[name] = {"error": str(e)[:200]}
        times = {n: [] for n in ctxs}
        names = list(ctxs)
        for r in range(rounds):
            for n in names[r % len(names):] + names[:r % len(names)]:  # each context first in turn
                L = ctxs[n]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                L.step(steps)
                L.sync()
                times[n].append((time.perf_counter() - t0) * 1e6 / steps)
        for n, L in ctxs.items():
            out[n] = {"us_per_step": round(statistics.median(times[n]), 3),
                      "us_per_step_rounds": [round(t, 3) for t in times[n]]}
            if n != "single":
                out[n]["schedule"] = L.schedule
    finally:
        for L in ctxs.values():
            L.close()
    base = out.get("single", {}).get("us_per_step")
    for name in ("rccl", "p2p"):
        if base and "us_per_step" in out.get(name, {}):
            out[name]["ratio_to_single"] = round(out[name]["us_per_step"] / base, 4)
    out["config"] = {"workload": "phi^4 256^3 fp32 as one z-slab with self-exchange (RCCL / P2P), one GPU",
                     "steps": steps, "rounds": rounds,
                     "method": "three open contexts timed in turn (the order rotating), medians of the rounds"}
    return out


def c1_phi4_32_record(a, local):
    """BASELINE configs[0] read literally: a 32^3 φ⁴ lattice, Δτ = 0.01, 1000
    Langevin steps driven through tauhost.o with taumain.py's 13-argument argv
    (SQ_MODEL=phi4 SQ_SHAPE=32x32x32: one frame of 1000 steps), its end-file
    field compared bit for bit with the same frame run through the library."""
    import tempfile
    import numpy as np
    from stochquant_amd import Phi4Lattice, langevin
    seed, loops, dtau = 0x5EED, 1000, 0.01
    with tempfile.TemporaryDirectory() as td:
        end = os.path.join(td, "end_phi4")
        perf = os.path.join(td, "perf.json")
        argv = langevin.tauhost_argv(32, 1.0, dtau, 1, 0, 1.0, local, 1, 0, loops, "0", end, 16)
        env = dict(os.environ, SQ_MODEL="phi4", SQ_SHAPE="32x32x32", SQ_SEED=str(seed), SQ_PERF_JSON=perf)
        t0 = time.perf_counter()
        r = langevin.run_tauhost(argv, cwd=td, timeout=120, env=env)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            return {"error": r.stderr.decode(errors="replace")[-300:]}
        with open(perf) as fh:
            pj = json.load(fh)
        fcli = np.load(end, allow_pickle=False)
    with Phi4Lattice((32, 32, 32), dtau=dtau, m2=1.0, lam=1.0, seed=seed, device=local, loops=loops) as L:
        L.init_field(float(np.sqrt(2.0 * dtau)))       # tauhost.o's start field (run_phi4)
        stable = L.run_frame()
        flib = L.download()
    return {"config": {"workload": "BASELINE configs[0] literally: 32^3 scalar phi^4, dt = 0.01, 1000 Langevin "
                                   "steps, through tauhost.o with taumain.py's argv (SQ_MODEL=phi4)",
                       "argv": argv[1:], "lattice": [32, 32, 32]},
            "value": pj.get("site_updates_per_s"), "unit": "site-updates/s (inside the frame)",
            "frame_seconds": pj.get("frame_seconds"), "process_wall_s": round(wall, 3),
            "stable": bool(stable), "tauhost_equals_library": bool(np.array_equal(fcli, flib))}


def noise_check(lat, world, shape, local, corrupt=False):
    """oracle_check_noise (collective): the C = 1 protocol on this rank's slab,
    the kernel it launched most, and the verdict against the oracle's digests
    in device-transcendental mode (verify.oracle_check_noise: the ranks' table
    digests first).  Returns (verdict, kernel)."""
    import torch.distributed as dist
    from stochquant_amd import verify
    lat.perf_reset()
    d = verify.run_oracle_protocol(lat, corrupt=corrupt, noise=True)
    kernel = lat.launch_info()["kernel"]
    td = verify.bm_tables_digest(verify.bm_tables(local))
    pairs = [None] * world
    if world > 1:
        dist.all_gather_object(pairs, (d, td))
    else:
        pairs = [(d, td)]
    return verify.oracle_check_noise([q[0] for q in pairs], [q[1] for q in pairs], shape, world), kernel


def c5_record(a, world, rank, local, watch):
    """BASELINE configs[4] / SURVEY §8d C5 in the same invocation: the 1024^3
    lattice strong-scaled over the job's ranks (z-slabs, deep-halo exchange
    overlapped with the interior on the second stream; one slab at N = 1),
    timed like the headline (settle, warm-up, --steps, max over ranks), with
    its own multi_rank_check, oracle_check and oracle_check_noise against the
    committed digests of 1024^3 at this N.  Collective: every rank runs it."""
    import torch.distributed as dist
    from stochquant_amd import verify
    L5 = 1024
    shape = (L5, L5, L5)
    lat, slab_path = make_lattice(a, shape, world, rank, local)
    try:
        lat.init_field(0.1)
        t, perf, settle, ssteps = measure(a, lat, world, slab_path, watch)
        sites_local = lat.nz_local * L5 * L5
        rl, _, _ = roofline(a, lat, L5, world, slab_path, t, perf, 1, sites_local)
        checks = {}
        for key, fn, cmp in (("multi_rank_check", verify.run_protocol, verify.check),
                             ("oracle_check", verify.run_oracle_protocol, verify.oracle_check)):
            d = fn(lat)
            digests = [None] * world
            if world > 1:
                dist.all_gather_object(digests, d)
            else:
                digests = [d]
            checks[key] = cmp(digests, shape, world)
        checks["oracle_check_noise"], checks["oracle_check_noise_kernel"] = noise_check(lat, world, shape, local)
        ghost = lat.ghost[0] if slab_path else None
        schedule = lat.schedule if slab_path else None
        nz_local = lat.nz_local
    finally:
        lat.close()
    value = float(L5 ** 3) * a.steps / t
    return {"config": {"workload": f"phi^4 3-D Langevin step, 1024^3 fp32 split over {world} GPU(s) (BASELINE "
                                   f"configs[4], strong scaling)", "lattice": list(shape),
                       "per_gpu": [L5, L5, nz_local], "ghost_depth": ghost, "block_schedule": schedule,
                       "dtau": a.dtau, "m2": 1.0, "lambda": 1.0},
            "value": value, "unit": "site-updates/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "settle_ms": round(settle, 1), "settle_steps": ssteps, "ms_per_step": t * 1e3 / a.steps,
            "scaling": "strong", "roofline": rl, **checks}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, rank_deadline(a)))
    rank = int(os.environ.get("RANK", "0"))
    from stochquant_amd import rankwatch
    # every rank reports its phase and ends itself at the deadline (rank 0 first
    # printing the error line with all ranks' phases): a hang in the first
    # cross-device comm set-up or exchange must not leave the driver without a line
    watch = rankwatch.Watch(rank, world, rank_deadline(a), METRIC)
    watch.on_sigterm()
    try:
        run(a, world, rank, watch)
    except Exception as e:   # one line with the cause instead of a bare traceback
        watch.fail(e)
        raise


def run(a, world, rank, watch):
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    a.gpus = world
    import torch
    import torch.distributed as dist
    from stochquant_amd import _lib, verify
    _lib.load()  # fail loudly if the HIP library is missing
    if world > 1:
        watch.phase("rendezvous")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one node by contract: RCCL's bootstrap over loopback (data moves over xGMI)
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if a.inject_error is not None and a.inject_error == rank:
        watch.phase("injected")
        raise RuntimeError("injected failure (--inject-error)")
    if a.inject_stall:
        r_s, sec = a.inject_stall.split(":")
        if int(r_s) == rank:
            watch.phase("stall")
            time.sleep(float(sec))
    if a.dry_run:
        watch.phase("dry_run")
        dry_run(a, world, rank, local, dist)
        if world > 1:
            dist.destroy_process_group()
        watch.finish()
        return
    torch.cuda.set_device(local)
    a.transport, a.transport_fallback = a.comm, None
    # RCCL's bring-up and exchanges give up after this (the library's default is
    # 300 s): short enough that a failed RCCL start still leaves the P2P
    # fallback and the timed run inside the rank deadline
    os.environ.setdefault("SQ_COMM_TIMEOUT_S", "90")
    L = a.size
    shape = (L, L, L) if a.strong else (L, L, L * world)
    watch.phase("comm_init", comm=a.comm, shape=list(shape))
    lat, slab_path = make_lattice(a, shape, world, rank, local)
    lat.init_field(0.1)
    t, perf, settle_ms, settle_steps = measure(a, lat, world, slab_path, watch)
    # sanity: the field stayed finite and bounded (no guard hits)
    m = lat.moments()
    sites_local = lat.nz_local * L * L
    total_updates = float(shape[0] * shape[1] * shape[2]) * a.steps
    value = total_updates / t
    nslabs = a.slabs if (world == 1 and a.comm == "loopback") else 1
    rl, _, fused = roofline(a, lat, L, world, slab_path, t, perf, nslabs, sites_local)
    achieved_wall = BYTES_PER_SITE * value / 1e9
    rl["frac_algorithmic_wall"] = round(achieved_wall / HBM_PEAK_GBPS, 4)
    rl["achieved_algorithmic_wall_GBps"] = round(achieved_wall, 1)
    # self-check (verify.py): the check protocol's slab digests against the
    # golden ones of a single-GPU run of the same global lattice, every rank
    check = "skipped"
    watch.phase("check")
    if not a.no_check and a.dtau == verify.CHECK_PARAMS["dtau"]:
        d = verify.run_protocol(lat, corrupt=(rank == a.corrupt_rank))
        digests = [None] * world
        if world > 1:
            dist.all_gather_object(digests, d)
        else:
            digests = [d]
        check = verify.check(digests, shape, world)
    # parity: the same lattice with the noise off from the
    # hash field, every rank's slab after CHECK_STEPS steps against the digests
    # the CPU oracle produced (tests/golden/oracle_slabs.json) -- on every N
    ocheck = "skipped"
    watch.phase("oracle_check")
    if not a.no_check and a.dtau == verify.CHECK_PARAMS["dtau"]:
        d = verify.run_oracle_protocol(lat, corrupt=(rank == a.corrupt_rank))
        digests = [None] * world
        if world > 1:
            dist.all_gather_object(digests, d)
        else:
            digests = [d]
        ocheck = verify.oracle_check(digests, shape, world)
    # the same protocol with the noise ON through the timed kernel instance
    # (VERDICT r5 next #6): digests against the oracle's in device-transcendental
    # mode, compared only when this device's Box-Muller tables are the ones the
    # committed digests were made with
    ncheck, nkernel = "skipped", None
    watch.phase("oracle_check_noise")
    if not a.no_check and a.dtau == verify.CHECK_PARAMS["dtau"]:
        ncheck, nkernel = noise_check(lat, world, shape, local, corrupt=(rank == a.corrupt_rank))
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
                               f"z-slab x{world} ({a.comm if world == 1 or a.comm == 'p2p' else a.transport}), halo "
                               + ("exchange in order on the interior stream between blocks"
                                  if (schedule or {}).get("exchange_in_order") else
                                  "exchange on stream B, interior on stream A"),
            },
            "transport_fallback": a.transport_fallback,
            "roofline": rl,
            "multi_rank_check": check,
            "oracle_check": ocheck,
            "oracle_check_protocol": (f"C = 0, verify.hash_field initial field, step counter 0, {verify.CHECK_STEPS} "
                                      f"steps through the same context (same kernels, slabs and exchanges); every "
                                      f"rank's slab digest vs the CPU oracle's (oracle/orc_phi4.c via "
                                      f"tests/golden/make_oracle_slabs.py -> tests/golden/oracle_slabs.json)"),
            "oracle_check_noise": ncheck,
            "oracle_check_noise_protocol": (f"C = 1, the same hash field and {verify.CHECK_STEPS} steps through the "
                                            f"same context (kernel {nkernel}); every rank's slab digest vs the CPU "
                                            f"oracle's in device-transcendental mode (the device's Box-Muller "
                                            f"tables, their blake2b checked first; tests/golden/make_oracle_slabs.py "
                                            f"--noise)"),
            "multi_rank_check_protocol": (f"init 0.1*normal, step counter 0, {verify.CHECK_STEPS} steps; every "
                                          f"rank's slab digest vs the golden single-GPU run "
                                          f"(stochquant_amd/golden_slabs.json)"),
            "hbm_copy_peak_GBps": copy,
            "field_check": {"rms": (m["sum2"] / sites_local) ** 0.5, "maxabs": m["maxabs"]},
        }
        if world == 1 and not a.no_cpu_baseline:
            watch.phase("cpu_baseline")
            out["cpu_baseline"] = cpu_baseline(L, a.dtau, a.cpu_seconds)
        else:
            out["cpu_baseline"] = None
    # the headline is complete: from here on a deadline or a hang in an optional
    # sub-record prints this line (marked incomplete) instead of an error line
    watch.set_partial(out if rank == 0 else {})
    # config C3 (BASELINE configs[2], 512^3 on one GPU) in the same invocation:
    # the same settle, warm-up and --steps, its own roofline and CPU sample
    if world == 1 and not a.strong and a.comm == "auto" and L == 256 and not a.no_c3:
        L3 = 512
        watch.phase("c3_512")
        lat3, _ = make_lattice(a, (L3, L3, L3), 1, 0, local)
        lat3.init_field(0.1)
        t3, perf3, settle3, ssteps3 = measure(a, lat3, 1, False)
        sites3 = L3 ** 3
        rl3, value3, _ = roofline(a, lat3, L3, 1, False, t3, perf3, 1, sites3)
        rl3["frac_algorithmic_wall"] = round(BYTES_PER_SITE * value3 / 1e9 / HBM_PEAK_GBPS, 4)
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
    # config C1 (BASELINE configs[0], the reference's own 1-D chain at 32,768 sites)
    if out is not None and world == 1 and not a.strong and a.comm == "auto" and L == 256 and not a.no_c1:
        watch.phase("c1_qm1d")
        try:
            out["c1_qm1d"] = c1_record(a, local)
        except Exception as e:  # the headline record stands without it
            out["c1_qm1d"] = {"error": str(e)[:300]}
    # the frame loop, the one-GPU slab path and the literal configs[0] (VERDICT r4
    # next #4, #5, #7), measured in the same invocation as the headline
    if out is not None and world == 1 and not a.strong and a.comm == "auto" and L == 256 and not a.no_extra:
        for key, fn in (("frames_256", frames_record), ("slab_1gpu", slab_record),
                        ("c1_phi4_32", c1_phi4_32_record)):
            watch.phase(key)
            try:
                out[key] = fn(a, local)
            except Exception as e:  # the headline record stands without it
                out[key] = {"error": str(e)[:300]}
    # config C5 (BASELINE configs[4]): 1024^3 strong-scaled over the same ranks
    if not a.strong and a.comm == "auto" and L == 256 and not a.no_c5:
        watch.phase("c5_1024")
        try:
            c5 = c5_record(a, world, rank, local, watch)
        except Exception as e:  # the headline record stands without it
            c5 = {"error": str(e)[:300]}
        if out is not None:
            out["c5_1024"] = c5
    if world > 1:
        watch.phase("teardown")
        dist.barrier()
        dist.destroy_process_group()
    watch.finish()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
