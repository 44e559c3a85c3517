"""Host-side mirror of the reference's interface for the Langevin path.

The reference exposes no Python API: `taumain.py:132` spawns `./tauhost.o`
with 13 positional arguments and parses its stdout.  This module offers that
same contract (`run_tauhost`, `parse_frame_line`) plus thin numpy wrappers of
the C ABI for the two models:

* `Qm1dChain`  -- tau_kernel.cl time_dev + the tauhost.c frame loop (fp64)
* `Phi4Lattice` -- the 3-D fp32 north-star extension (slab / multi-GPU)

Everything computes on the MI355X through libstochquant.so; nothing here has a
CPU path.
"""
import ctypes
import io
import os
import subprocess

import numpy as np

from . import _lib
from ._lib import (SQ_COMM_LOOPBACK, SQ_COMM_NONE, SQ_COMM_P2P, SQ_COMM_RCCL, SQ_MODEL_PHI4, SQ_MODEL_QM1D, SQ_ORDER_JACOBI,
                   SQ_ORDER_SERIAL)

_DP = ctypes.POINTER(ctypes.c_double)
_FP = ctypes.POINTER(ctypes.c_float)


def _dptr(a):
    return a.ctypes.data_as(_DP)


def _fptr(a):
    return a.ctypes.data_as(_FP)


class _Ctx:
    def __init__(self, params):
        self._h = ctypes.c_void_p()
        _lib.call("sq_create", ctypes.byref(params), ctypes.byref(self._h))
        self.params = params

    def close(self):
        if self._h:
            _lib.call("sq_destroy", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # shared controls ------------------------------------------------------
    @property
    def dtau(self):
        d = ctypes.c_double()
        _lib.call("sq_get_dtau", self._h, ctypes.byref(d))
        return d.value

    @dtau.setter
    def dtau(self, v):
        _lib.call("sq_set_dtau", self._h, float(v))

    @property
    def step_counter(self):
        s = ctypes.c_ulonglong()
        _lib.call("sq_get_step", self._h, ctypes.byref(s))
        return s.value

    @step_counter.setter
    def step_counter(self, v):
        _lib.call("sq_set_step", self._h, int(v))

    def run_frame(self):
        """`loops` steps + stability check + rollback + Δτ control; returns True if stable."""
        st = ctypes.c_int()
        _lib.call("sq_run_frame", self._h, ctypes.byref(st))
        return st.value == 1

    def run_frames(self, n):
        """n frames back to back (sq_run_frames: for phi^4 the verdict, rollback
        and Δτ controller stay on the device); returns (stable bool array, Δτ
        after each frame)."""
        import numpy as np
        st = np.zeros(max(n, 1), dtype=np.int32)
        dt = np.zeros(max(n, 1), dtype=np.float64)
        _lib.call("sq_run_frames", self._h, int(n), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                  dt.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return st[:n] == 1, dt[:n]

    def set_profiling(self, mode=1):
        """0 off; 1 every step kernel timed by dispatch events; 2 one event pair per step() call."""
        _lib.call("sq_set_profiling", self._h, int(mode))

    def perf(self):
        p = _lib.SqPerf()
        _lib.call("sq_perf", self._h, ctypes.byref(p))
        return {k: getattr(p, k) for k, _ in p._fields_}

    def perf_reset(self):
        _lib.call("sq_perf_reset", self._h)

    def sync(self):
        _lib.call("sq_sync", self._h)

    def set_noise(self, C):
        """Noise amplitude C of the open context (C = 0: drift only, deterministic)."""
        _lib.call("sq_set_noise", self._h, float(C))
        self.params.C = float(C)


class Qm1dChain(_Ctx):
    """The reference's 1-D chain: N sites (Δt spacing), potID 0 or 3, noise C,
    `loops` steps per frame (tauhost.c argv[1..10] meaning)."""

    def __init__(self, N, deltat, deltatau, pot=3, C=1.0, loops=1000, seed=0x5EED, device=0,
                 adapt_dtau=True, ordering="jacobi", lcg_seed=None):
        p = _lib.default_params()
        p.model = SQ_MODEL_QM1D
        p.dims[0] = int(N)
        p.deltat = float(deltat)
        p.deltatau = float(deltatau)
        p.pot = int(pot)
        p.C = float(C)
        p.loops = int(loops)
        p.seed = int(seed)
        p.device = int(device)
        p.adapt_dtau = 1 if adapt_dtau else 0
        super().__init__(p)
        self.N = int(N)
        if ordering != "jacobi":
            self.set_ordering(ordering)
        if lcg_seed is not None:
            self.lcg_seed = lcg_seed

    def set_ordering(self, ordering):
        """"jacobi" (Philox noise, the fast path) or "serial" (the reference's
        Gauss-Seidel order with its shared-seed LCG, SQ_ORDER_SERIAL)."""
        _lib.call("sq_qm1d_set_ordering", self._h, {"jacobi": SQ_ORDER_JACOBI, "serial": SQ_ORDER_SERIAL}[ordering])

    @property
    def lcg_seed(self):
        v = ctypes.c_ulonglong()
        _lib.call("sq_qm1d_get_lcg_seed", self._h, ctypes.byref(v))
        return v.value

    @lcg_seed.setter
    def lcg_seed(self, v):
        _lib.call("sq_qm1d_set_lcg_seed", self._h, int(v))

    def inject_noise(self, xi):
        """Draws for the next serial frame, in call order (round*(N+1) + item)."""
        xi = np.ascontiguousarray(xi, dtype=np.float64)
        _lib.call("sq_qm1d_inject_noise", self._h, _dptr(xi), xi.size)

    @property
    def noise_consumed(self):
        v = ctypes.c_ulonglong()
        _lib.call("sq_qm1d_noise_consumed", self._h, ctypes.byref(v))
        return v.value

    def upload(self, f, x=None, xx0=None, omega=0.0, runs=0):
        f = np.ascontiguousarray(f, dtype=np.float64)
        x = np.zeros(self.N) if x is None else np.ascontiguousarray(x, dtype=np.float64)
        xx0 = np.zeros(self.N) if xx0 is None else np.ascontiguousarray(xx0, dtype=np.float64)
        if f.shape != (self.N,) or x.shape != (self.N,) or xx0.shape != (self.N,):
            raise ValueError("state arrays must have N entries")
        _lib.call("sq_upload", self._h, _dptr(f), _dptr(x), _dptr(xx0), float(omega), int(runs))

    def download(self):
        f, x, xx0 = np.empty(self.N), np.empty(self.N), np.empty(self.N)
        om = ctypes.c_double()
        runs = ctypes.c_long()
        _lib.call("sq_download", self._h, _dptr(f), _dptr(x), _dptr(xx0), ctypes.byref(om), ctypes.byref(runs))
        return {"f": f, "x": x, "xx0": xx0, "omega": om.value, "runs": runs.value}

    @property
    def scan(self):
        e, v, t = ctypes.c_int(), ctypes.c_double(), ctypes.c_ulonglong()
        _lib.call("sq_qm1d_get_scan", self._h, ctypes.byref(e), ctypes.byref(v), ctypes.byref(t))
        return {"lrgEl": e.value, "lrgVl": v.value, "tick": t.value}

    def set_scan(self, lrgEl, lrgVl, tick):
        _lib.call("sq_qm1d_set_scan", self._h, int(lrgEl), float(lrgVl), int(tick))

    def xavg(self):
        """xavg = xx0 - x * x[mid] (tauhost.c:519-521)."""
        out = np.empty(self.N)
        _lib.call("sq_correlator", self._h, _dptr(out), self.N)
        return out


class Phi4Lattice(_Ctx):
    """Periodic 3-D φ⁴ lattice (Lx, Ly, Lz) in fp32, V = m²/2 φ² + λ/24 φ⁴.

    comm="none"     one slab, z wraps in-kernel
    comm="loopback" `nslabs` slabs on one device, halos by D2D copies
    comm="rccl"     one slab per process (rank / nranks), halos over RCCL;
                    `comm_id` from `unique_id()` on rank 0
    comm="p2p"      one slab per process, halos pulled from the neighbours'
                    memory (IPC peer pointers), no RCCL; every rank passes
                    all ranks' `p2p_handle()` blobs, in rank order, to
                    `p2p_connect` before stepping (`connect_p2p` does it over
                    a torch.distributed group)
    """

    def __init__(self, shape, dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED, device=0, comm="none",
                 nslabs=1, nranks=1, rank=0, comm_id=None, clamp=1000.0, loops=100, C=1.0,
                 adapt_dtau=True):
        p = _lib.default_params()
        p.model = SQ_MODEL_PHI4
        for i in range(3):
            p.dims[i] = int(shape[i])
        p.deltatau = float(dtau)
        p.m2 = float(m2)
        p.lambda_ = float(lam)
        p.seed = int(seed)
        p.device = int(device)
        p.clamp = float(clamp)
        p.loops = int(loops)
        p.C = float(C)
        p.adapt_dtau = 1 if adapt_dtau else 0
        p.comm = {"none": SQ_COMM_NONE, "loopback": SQ_COMM_LOOPBACK, "rccl": SQ_COMM_RCCL, "p2p": SQ_COMM_P2P}[comm]
        p.nslabs = int(nslabs)
        p.nranks = int(nranks)
        p.rank = int(rank)
        if comm_id is not None:
            b = bytes(comm_id)
            ctypes.memmove(p.comm_id, b, min(len(b), 128))
        super().__init__(p)
        self.shape = tuple(int(s) for s in shape)
        nz, z0 = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.call("sq_slab", self._h, ctypes.byref(nz), ctypes.byref(z0))
        self.nz_local, self.z0 = nz.value, z0.value

    @property
    def local_shape(self):
        return (self.nz_local, self.shape[1], self.shape[0])  # numpy order: z, y, x

    def step(self, n=1):
        _lib.call("sq_step", self._h, int(n))

    def upload(self, phi):
        a = np.ascontiguousarray(phi, dtype=np.float32)
        if a.size != int(np.prod(self.local_shape)):
            raise ValueError(f"field must have {self.local_shape} entries")
        _lib.call("sq_upload_field", self._h, _fptr(a), a.size)

    def download(self):
        a = np.empty(self.local_shape, dtype=np.float32)
        _lib.call("sq_download_field", self._h, _fptr(a), a.size)
        return a

    def init_field(self, amp):
        _lib.call("sq_init_field", self._h, float(amp))

    def init_field_hash(self, amp, key):
        """phi = amp * (top 24 bits of splitmix64(global index ^ key) - 2^23) / 2^23 (sq_init_field_hash)."""
        _lib.call("sq_init_field_hash", self._h, float(amp), int(key))

    def moments(self):
        out = np.zeros(3)
        _lib.call("sq_moments", self._h, _dptr(out))
        return {"sum": out[0], "sum2": out[1], "maxabs": out[2]}

    @property
    def tile(self):
        """(lanes per x segment, rows per lane, z planes per wave, float4 segments per lane)."""
        out = (ctypes.c_int * 4)()
        _lib.call("sq_phi4_tile", self._h, out)
        return tuple(out)

    @property
    def kernel_name(self):
        """The step kernel instance as rocprofv3 names it, plus the z-chunk."""
        buf = ctypes.create_string_buffer(160)
        _lib.call("sq_phi4_kernel", self._h, buf, len(buf))
        return buf.value.decode()

    def launch_info(self):
        """The step kernel launched most often since perf_reset(): {"kernel": template
        instance as rocprofv3 names it, "grid": threads, "launches": n}."""
        buf = ctypes.create_string_buffer(160)
        g, n = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.call("sq_phi4_launch_info", self._h, buf, len(buf), ctypes.byref(g), ctypes.byref(n))
        return {"kernel": buf.value.decode(), "grid": g.value, "launches": n.value}

    @property
    def ghost(self):
        """(active, allocated) ghost-zone depth of a slab decomposition; (0, 0) for one periodic slab."""
        a, b = ctypes.c_int(), ctypes.c_int()
        _lib.call("sq_phi4_ghost", self._h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    @property
    def schedule(self):
        """{"ghost", "core_pairs", "rims_b", "edge_first", "tuned", "exchange_in_order", "kstaged"} of a slab
        decomposition's block schedule (sq_phi4_schedule, sq_phi4_edge_first, sq_phi4_exchange_stream)."""
        k, b, t, e = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.call("sq_phi4_schedule", self._h, ctypes.byref(k), ctypes.byref(b), ctypes.byref(t))
        _lib.call("sq_phi4_edge_first", self._h, ctypes.byref(e))
        a, ks = ctypes.c_int(), ctypes.c_int()
        _lib.call("sq_phi4_exchange_stream", self._h, ctypes.byref(a), ctypes.byref(ks))
        return {"ghost": self.ghost[0], "core_pairs": k.value, "rims_b": bool(b.value), "edge_first": bool(e.value),
                "tuned": bool(t.value), "exchange_in_order": bool(a.value), "kstaged": bool(ks.value)}

    def save(self, path):
        """Binary checkpoint: <path> (.npy float32 (nz, Ly, Lx)) + <path>.json (step, dtau, seed, z0)."""
        _lib.call("sq_save_field", self._h, os.fsencode(path))

    def load(self, path, restore_counters=True):
        _lib.call("sq_load_field", self._h, os.fsencode(path), 1 if restore_counters else 0)

    def stability(self, n=None):
        """The frame stability heuristic's state: {"T", "V", "fired" (step of the
        last frame it fired at, -1 none), "M", "D", "A" (that frame's per-step
        records)} -- DESIGN.md §7."""
        n = self.params.loops if n is None else int(n)
        st = np.zeros(2)
        fired = ctypes.c_int()
        M, D, A = (np.zeros(n, dtype=np.float32) for _ in range(3))
        _lib.call("sq_phi4_stability", self._h, _dptr(st), ctypes.byref(fired), _fptr(M), _fptr(D), _fptr(A), n)
        return {"T": st[0], "V": st[1], "fired": fired.value, "M": M, "D": D, "A": A}

    def block_stamps(self, cap=1 << 16):
        """Run 2 steps (one fused launch) with per-block clock stamps; returns
        (start, end) int64 arrays in ticks of the 100 MHz constant clock."""
        a = np.zeros(2 * cap, dtype=np.uint64)
        nb = ctypes.c_int()
        _lib.call("sq_phi4_block_stamps", self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), int(cap),
                  ctypes.byref(nb))
        a = a[:2 * nb.value].astype(np.int64)
        return a[0::2], a[1::2]

    def block_clocks(self, cap=1 << 16):
        """The last block_stamps launch's shader-clock counter (s_memtime) at each
        block's start and end: (start, end) int64 arrays in shader cycles."""
        a = np.zeros(2 * cap, dtype=np.uint64)
        nb = ctypes.c_int()
        _lib.call("sq_phi4_block_clocks", self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), int(cap),
                  ctypes.byref(nb))
        a = a[:2 * nb.value].astype(np.int64)
        return a[0::2], a[1::2]

    def set_stability(self, T, V):
        _lib.call("sq_phi4_set_stability", self._h, float(T), float(V))

    def correlator(self, n=None):
        n = self.shape[2] if n is None else int(n)
        out = np.empty(n)
        _lib.call("sq_correlator", self._h, _dptr(out), n)
        return out

    def p2p_handle(self):
        """This rank's SQ_COMM_P2P handle blob (bytes) for the other ranks."""
        buf = (ctypes.c_ubyte * _lib.SQ_P2P_HANDLE_BYTES)()
        _lib.call("sq_p2p_handle", self._h, buf)
        return bytes(buf)

    def p2p_connect(self, blobs):
        """Map the peers of an SQ_COMM_P2P context: `blobs` = every rank's p2p_handle(), in rank order."""
        n = _lib.SQ_P2P_HANDLE_BYTES
        if any(len(b) != n for b in blobs):
            raise ValueError(f"every handle blob has {n} bytes")
        buf = (ctypes.c_ubyte * (n * len(blobs))).from_buffer_copy(b"".join(blobs))
        _lib.call("sq_p2p_connect", self._h, buf, len(blobs))


def connect_p2p(lat, group=None):
    """All-gather the ranks' P2P handle blobs over torch.distributed and connect."""
    import torch.distributed as dist
    blobs = [None] * dist.get_world_size(group)
    dist.all_gather_object(blobs, lat.p2p_handle(), group=group)
    lat.p2p_connect(blobs)


def unique_id():
    """RCCL unique id (128 bytes) for SQ_COMM_RCCL contexts."""
    buf = (ctypes.c_ubyte * 128)()
    _lib.call("sq_comm_unique_id", buf)
    return bytes(buf)


# --------------------------------------------------------------------------
# Process/CLI contract of the reference (taumain.py:132 -> tauhost.o)
# --------------------------------------------------------------------------
TAUHOST_ARGS = ("n", "deltat", "deltatau", "frames", "potID", "c", "device", "rpf", "intime",
                "loops", "inputf", "outputf", "acco")


def tauhost_argv(n, deltat, deltatau, frames, potID, c, device, rpf, intime, loops, inputf, outputf,
                 acco, exe=None):
    """argv exactly as taumain.py:132 builds it (every value passed through str())."""
    exe = exe or _lib.TAUHOST_PATH
    return [exe] + [str(v) for v in (n, deltat, deltatau, frames, potID, c, device, rpf, intime, loops,
                                     inputf, outputf, acco)]


def run_tauhost(argv, cwd=None, timeout=600, env=None):
    """Run the drop-in executable; returns CompletedProcess with bytes stdout."""
    if not os.path.exists(argv[0]):
        raise _lib.StochQuantUnavailable(f"{argv[0]} not built")
    return subprocess.run(argv, cwd=cwd, capture_output=True, timeout=timeout, env=env)


def parse_frame_line(line):
    """taumain.py:30-41: np.genfromtxt(delimiter='|'); last two fields Δτ, percent."""
    tmp = np.genfromtxt(io.BytesIO(line.strip()), delimiter="|")
    return {"y": tmp[:-2], "dtau": tmp[-2], "percent": tmp[-1]}
