"""Per-rank phase reports and a deadline for multi-rank runs (bench.py).

Every rank writes its current phase ("rendezvous", "comm_init", "trial_blocks",
"timed", "check", ...) into `<dir>/rank<r>.json`.  A watchdog thread in each
rank enforces one deadline for the whole run: when it passes, rank 0 prints ONE
JSON line with "error" and every rank's last phase (so a hang in the first
xGMI ncclCommInitRank or a peer-memory exchange leaves a diagnosis, not just a
time-limit kill), and every rank ends itself with exit code 3.  `os._exit`
ends the process without unwinding the thread that is stuck in a device call;
the runtime releases the device queues at process exit.

The parent that spawned the ranks (bench.py's spawn_ranks) applies the same
deadline plus a grace period from outside, for a rank whose watchdog cannot
run (ctypes releases the interpreter lock during library calls, so a rank
stuck in one still runs its watchdog; a rank stuck elsewhere may not).
"""
import json
import os
import threading
import time

EXIT_DEADLINE = 3


def phase_dir(port=None):
    """The directory the ranks of one job share (keyed by the rendezvous port)."""
    d = os.environ.get("SQ_PHASE_DIR")
    if d:
        return d
    port = port or os.environ.get("MASTER_PORT", "0")
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"sq_ranks_{os.getuid()}_{port}")


def read_phases(d, world):
    out = {}
    now = time.time()
    for r in range(world):
        try:
            with open(os.path.join(d, f"rank{r}.json")) as fh:
                rec = json.load(fh)
            rec["age_s"] = round(now - rec.pop("t", now), 1)
            out[str(r)] = rec
        except (OSError, ValueError):
            out[str(r)] = {"phase": "no report"}
    return out


def error_line(metric, world, deadline_s, phases, why):
    return json.dumps({"metric": metric, "value": None, "n_gpus": world, "error": why,
                       "deadline_s": deadline_s, "rank_phases": phases})


class Watch:
    """Phase reporter + deadline for one rank."""

    def __init__(self, rank, world, deadline_s, metric, d=None, on_expire=None):
        self.rank, self.world, self.deadline_s, self.metric = rank, world, float(deadline_s), metric
        self.dir = d or phase_dir()
        os.makedirs(self.dir, exist_ok=True)
        self.t0 = time.time()
        self.phase_name = None
        self.partial = None      # rank 0: the bench line once its headline part is complete (set_partial)
        self.done = threading.Event()
        self.on_expire = on_expire or self._expire
        self.phase("start")
        if self.deadline_s > 0:
            threading.Thread(target=self._run, daemon=True, name="sq-rank-deadline").start()

    def phase(self, name, **info):
        if name != "error":
            self.phase_name = name
        rec = {"rank": self.rank, "phase": name, "t": time.time(), "elapsed_s": round(time.time() - self.t0, 2)}
        rec.update(info)
        tmp = os.path.join(self.dir, f".rank{self.rank}.json.tmp")
        with open(tmp, "w") as fh:
            json.dump(rec, fh)
        os.replace(tmp, os.path.join(self.dir, f"rank{self.rank}.json"))

    def set_partial(self, line):
        """The run's line with its headline complete (a dict, still growing as
        the optional sub-records are added).  From here on a deadline or a
        SIGTERM prints it, marked incomplete, instead of the error line, and
        the rank exits 0: a hang in an optional sub-record (a second
        communicator, the 1024^3 strong-scaling record) does not cost the
        headline."""
        self.partial = line

    def _print_partial(self, why):
        d = dict(self.partial)
        d["incomplete"] = {"phase": self.phase_name, "why": why,
                           "rank_phases": read_phases(self.dir, self.world)}
        print(json.dumps(d), flush=True)

    def fail(self, exc):
        """This rank raised: record it for the others' reports; rank 0 prints the line."""
        msg = f"{type(exc).__name__}: {exc}"[:400]
        self.phase("error", error=msg, failed_in=self.phase_name)
        if self.rank == 0:
            print(error_line(self.metric, self.world, self.deadline_s, read_phases(self.dir, self.world),
                             f"rank 0 failed: {msg}"), flush=True)
        self.done.set()

    def on_sigterm(self):
        """Rank 0 killed by the launcher (torch.distributed.run ends every rank
        once one has failed): print the line with every rank's phase first."""
        import signal

        def handler(signum, frame):
            why = f"rank {self.rank} terminated (signal {signum}) in phase '{self.phase_name}'"
            if not self.done.is_set():
                self.done.set()
                if self.partial is not None:
                    self._print_partial(why)
                    os._exit(0)
                print(error_line(self.metric, self.world, self.deadline_s, read_phases(self.dir, self.world),
                                 why), flush=True)
            os._exit(128 + signum)
        if self.rank == 0:
            signal.signal(signal.SIGTERM, handler)

    def finish(self):
        self.phase("done")
        self.done.set()

    def _run(self):
        if self.done.wait(self.deadline_s):
            return
        self.on_expire(self)

    def _expire(self, _self):
        if self.partial is not None:
            # rank 0 holds the completed headline: print it, every rank exits 0
            if self.rank == 0:
                self._print_partial(f"rank deadline of {self.deadline_s:.0f} s passed in an optional sub-record")
            os._exit(0)
        if self.rank == 0:
            phases = read_phases(self.dir, self.world)
            print(error_line(self.metric, self.world, self.deadline_s, phases,
                             f"rank deadline of {self.deadline_s:.0f} s passed; rank 0 in phase "
                             f"'{self.phase_name}'"), flush=True)
        os._exit(EXIT_DEADLINE)
