"""Headless mirror of the reference's Python caller, taumain.py.

taumain.py (the reference's only user-facing program) picks a preset
(taumain.py:91-110), spawns `./tauhost.o` with 13 positional arguments
(:112-132), and a reader thread parses every stdout line with
`np.genfromtxt(BytesIO(line.strip()), delimiter="|")`, keeping the last two
fields as (Δτ, percent) and queueing the rest, log|xavg_i| for i = 1..N-1, for
the plot (:17-48).  The matplotlib animation (:50-88) is a GUI and stays out
of scope; everything the plot consumes is produced here, against the
MI355X drop-in executable.

    from stochquant_amd.driver import PRESETS, TauhostRun
    with TauhostRun("double_well", frames=200) as run:
        for fr in run:                    # one dict per printed frame
            y, dtau, percent = fr["y"], fr["dtau"], fr["percent"]
"""
import os
import subprocess
import threading
from queue import Queue

from . import _lib
from .langevin import parse_frame_line, tauhost_argv

# taumain.py:91-110, verbatim values
PRESETS = {
    "harmosc": {"dtau": .3, "Nt": 100, "dt": .1, "potID": 0, "theoVal": 20., "c": 1., "filename": "HarmOsc.txt"},
    "double_well": {"dtau": .002, "Nt": 200, "dt": .02, "potID": 3, "theoVal": 10, "c": 1.,
                    "filename": "V0_2e_0-8.txt"},
}

# taumain.py:111-126
DEFAULTS = {"entw": 5000, "device": 2, "rpf": 1, "intime": 0, "loops": 1000, "acco": 40}


def preset_argv(name, frames=None, loops=None, device=None, rpf=None, start="0", end=None, acco=None,
                exe=None):
    """The argv taumain.py:132 builds for `name` (start file "0" = fresh start,
    end file = the preset's filename, as taumain.py:123-126)."""
    p = PRESETS[name]
    d = DEFAULTS
    return tauhost_argv(p["Nt"], p["dt"], p["dtau"], d["entw"] if frames is None else frames, p["potID"], p["c"],
                        d["device"] if device is None else device, d["rpf"] if rpf is None else rpf,
                        d["intime"], d["loops"] if loops is None else loops, start,
                        p["filename"] if end is None else end, d["acco"] if acco is None else acco, exe=exe)


class TauhostRun:
    """Spawn the executable as taumain.py does and iterate its parsed frames.

    A reader thread (taumain.py's dataThread) drains stdout line by line into a
    queue, so a slow consumer never blocks the GPU process on a full pipe;
    iteration yields {"y", "dtau", "percent"} per printed frame and ends when
    the process exits.  `returncode`, `stderr` and `last` (the last frame) are
    set after the iteration finishes or `wait()` returns."""

    def __init__(self, preset, cwd=None, env=None, exe=None, **kw):
        self.argv = preset_argv(preset, exe=exe, **kw)
        self.n = PRESETS[preset]["Nt"]
        self.cwd = cwd
        self.env = env
        self.proc = None
        self.q = Queue()
        self.last = None
        self.returncode = None
        self.stderr = b""

    def __enter__(self):
        if not os.path.exists(self.argv[0]):
            raise _lib.StochQuantUnavailable(f"{self.argv[0]} not built")
        self.proc = subprocess.Popen(self.argv, cwd=self.cwd, env=self.env, stdout=subprocess.PIPE,
                                     stderr=subprocess.PIPE, bufsize=0)
        self._t = threading.Thread(target=self._reader, daemon=True)
        self._t.start()
        return self

    def _reader(self):
        for line in iter(self.proc.stdout.readline, b""):
            if line.strip():
                self.q.put(parse_frame_line(line))
        self.q.put(None)

    def __iter__(self):
        while True:
            fr = self.q.get()
            if fr is None:
                break
            if fr["y"].size != self.n - 1:
                raise ValueError(f"frame line with {fr['y'].size} values, expected {self.n - 1}")
            self.last = fr
            yield fr
        self.wait()

    def wait(self, timeout=None):
        if self.proc is not None and self.returncode is None:
            self.returncode = self.proc.wait(timeout=timeout)
            self.stderr = self.proc.stderr.read()
            self._t.join(timeout=5)
        return self.returncode

    def __exit__(self, *exc):
        if self.proc is not None and self.proc.poll() is None:
            self.proc.kill()
        if self.proc is not None:
            self.wait()
            self.proc.stdout.close()
            self.proc.stderr.close()
        return False
