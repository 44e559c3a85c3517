"""bench.py's launch paths on a CPU host (--dry-run: ranks, process group and
schedule, no device): run bare with --gpus N it spawns its N rank processes
itself (the driver's scaling runs need no torchrun), under a launcher
(RANK / WORLD_SIZE set) it is one rank; rank 0 relays the single JSON line."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_ranks(n):
    d = _run(["--gpus", str(n), "--dry-run"])
    assert d["dry_run"] and d["n_gpus"] == n
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(n)) and [r["local_rank"] for r in ranks] == list(range(n))
    # weak scaling: 256^3 per rank, contiguous slabs covering 256 n planes
    assert [r["slab"] for r in ranks] == [[256 * k, 256 * (k + 1)] for k in range(n)]
    assert all(r["plan"][0] == "exchange" and "pair" in r["plan"] for r in ranks)


def test_bench_strong_split():
    d = _run(["--gpus", "2", "--dry-run", "--strong", "--size", "64"])
    assert [r["slab"] for r in sorted(d["ranks"], key=lambda r: r["rank"])] == [[0, 32], [32, 64]]


def test_bench_single_rank_under_a_launcher():
    """RANK / WORLD_SIZE present (torch.distributed.run): no spawning."""
    d = _run(["--dry-run"], env={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert d["n_gpus"] == 1 and d["ranks"][0]["plan"] is None


def _run_rc(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "SQ_PHASE_DIR"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def test_stalled_rank_ends_the_run_with_an_error_line():
    """One rank stalls after the rendezvous (VERDICT r3 next #2a): rank 0's
    deadline fires while it waits in the collective, it prints ONE JSON line
    with "error" and every rank's last phase, and the run exits 3 within the
    deadline (not at the driver's time limit)."""
    import time
    t0 = time.time()
    r = _run_rc(["--gpus", "2", "--dry-run", "--inject-stall", "1:90", "--rank-timeout", "6"])
    dt = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and "deadline" in d["error"] and d["n_gpus"] == 2
    assert d["rank_phases"]["1"]["phase"] == "stall" and d["rank_phases"]["0"]["phase"] == "dry_run"
    assert dt < 60, dt


def test_stalled_rank_under_a_launcher(tmp_path):
    """Launched as one rank by torch.distributed.run (no spawning parent): the
    rank's own watchdog still prints the line and exits 3; a rank that never
    reported shows as "no report"."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = {"RANK": "0", "WORLD_SIZE": "2", "LOCAL_RANK": "0", "SQ_PHASE_DIR": str(tmp_path),
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}
    # rank 1 never starts: rank 0 waits in the rendezvous until its deadline
    r = _run_rc(["--dry-run", "--rank-timeout", "5"], env=env)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["rank_phases"]["0"]["phase"] == "rendezvous" and d["rank_phases"]["1"]["phase"] == "no report"


def test_failing_rank_reports_its_error():
    """A rank that raises (after the rendezvous) ends the spawned run at once:
    the parent terminates the others, and rank 0's line carries the failed
    rank's phase and message."""
    r = _run_rc(["--gpus", "2", "--dry-run", "--inject-error", "1", "--rank-timeout", "60"])
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])
    d = json.loads(lines[0])
    # rank 0 either is terminated by the parent or first sees its collective
    # fail (the peer's socket closed); both lines name rank 1's error
    assert d["value"] is None and ("terminated" in d["error"] or "rank 0 failed" in d["error"])
    assert d["rank_phases"]["1"]["phase"] == "error" and "injected" in d["rank_phases"]["1"]["error"]


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_default_transport():
    """The driver's N > 1 path end to end on a one-GPU box: bench.py spawns two
    ranks on GPU 0 with the default transport.  RCCL refuses two ranks on one
    device, so the ranks must agree to fall back to P2P together (bench.py
    open_with_fallback), run, and pass the multi-rank golden-digest check."""
    d = _run(["--gpus", "2", "--same-device", "--steps", "20", "--warmup", "5", "--no-c3", "--no-c1",
              "--no-cpu-baseline", "--rank-timeout", "200"], timeout=280)
    assert d["n_gpus"] == 2 and d["value"] and d["value"] > 0
    assert d["multi_rank_check"] == "pass"
    par = d["config"]["parallelism"]
    if d["transport_fallback"] is not None:
        assert "(p2p)" in par
    else:
        assert "(rccl)" in par


def test_deadline_after_the_headline_prints_the_partial_line(tmp_path):
    """Once the headline is complete (Watch.set_partial), a deadline in an
    optional sub-record prints that line marked "incomplete" and every rank
    exits 0 -- a hang in, e.g., the 1024^3 strong-scaling record does not cost
    the headline; before it, the error line and exit 3 as before."""
    import subprocess
    import sys
    code = ("import sys, time, json; sys.path.insert(0, %r)\n"
            "from stochquant_amd import rankwatch\n"
            "w = rankwatch.Watch(int(sys.argv[1]), 2, 2.0, 'm', d=%r)\n"
            "if sys.argv[2] == '1': w.set_partial({'metric': 'm', 'value': 1.5} if sys.argv[1] == '0' else {})\n"
            "w.phase('c5_1024')\n"
            "time.sleep(30)\n") % (ROOT, str(tmp_path))
    for rank in ("0", "1"):
        for partial in ("1", "0"):
            r = subprocess.run([sys.executable, "-c", code, rank, partial], capture_output=True, text=True, timeout=60)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if partial == "1":
                assert r.returncode == 0, r.stderr
                if rank == "0":
                    d = json.loads(lines[0])
                    assert d["value"] == 1.5 and d["incomplete"]["phase"] == "c5_1024", d
                else:
                    assert lines == []
            else:
                assert r.returncode == 3
                if rank == "0":
                    assert json.loads(lines[0])["value"] is None
