"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker (or the timed CPU baseline).
The product never routes through it.  See sq_oracle.h for what each
restatement follows in the reference.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
CLI = os.path.join(HERE, "orc_tauhost")

_D = ctypes.POINTER(ctypes.c_double)
_F = ctypes.POINTER(ctypes.c_float)
_U32 = ctypes.POINTER(ctypes.c_uint32)


class Qm1d(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int), ("pot", ctypes.c_int), ("loops", ctypes.c_int),
        ("a", ctypes.c_double), ("c", ctypes.c_double), ("dtau", ctypes.c_double),
        ("seed", ctypes.c_uint64), ("tick", ctypes.c_uint64), ("runs", ctypes.c_int),
        ("f", _D), ("x", _D), ("xx0", _D), ("nf", _D), ("nx", _D), ("nxx0", _D),
        ("omega", ctypes.c_double), ("nomega", ctypes.c_double),
        ("lrgEl", ctypes.c_int), ("lrgVl", ctypes.c_double),
        ("stable", ctypes.c_int), ("steps_done", ctypes.c_int),
    ]


class SerialDev(ctypes.Structure):
    """orc_serial_dev: the reference's device buffers + kernel scalars (serial order)."""
    _fields_ = [
        ("N", ctypes.c_int), ("pot", ctypes.c_int), ("loops", ctypes.c_int),
        ("a", ctypes.c_double), ("c", ctypes.c_double),
        ("f", _D), ("x", _D), ("xx0", _D), ("nf", _D), ("nx", _D), ("nxx0", _D),
        ("omega", ctypes.c_double), ("seed", ctypes.c_uint64), ("stable", ctypes.c_int),
        ("dtau", ctypes.c_double), ("lrgEl", ctypes.c_int), ("lrgVl", ctypes.c_double),
        ("runs", ctypes.c_int),
    ]


class Phi4(ctypes.Structure):
    _fields_ = [
        ("Lx", ctypes.c_int), ("Ly", ctypes.c_int), ("Lz", ctypes.c_int),
        ("h", ctypes.c_float), ("m2", ctypes.c_float), ("lam", ctypes.c_float), ("clampv", ctypes.c_float),
        ("seed", ctypes.c_uint64), ("C", ctypes.c_double),
    ]


_lib = None


def build():
    r = subprocess.run(["make", "-C", HERE, "-j4"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stdout + r.stderr)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_philox4x32_10.argtypes = [_U32, _U32, _U32]
        L.orc_normals4.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, _F]
        L.orc_xcl.restype = ctypes.c_double
        L.orc_xcl.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.orc_intconst.restype = ctypes.c_double
        L.orc_intconst.argtypes = [ctypes.c_int]
        L.orc_qm1d_frame.argtypes = [ctypes.POINTER(Qm1d)]
        L.orc_serial_launch.argtypes = [ctypes.POINTER(SerialDev)]
        L.orc_ref_noise_stream.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _D, _U32, _U32,
                                           ctypes.POINTER(ctypes.c_uint64)]
        L.orc_libm_f32.argtypes = [ctypes.c_int, _F, _F, ctypes.c_longlong]
        L.orc_set_bm_tables.argtypes = [_F]
        L.orc_phi4_step.argtypes = [ctypes.POINTER(Phi4), _F, _F, ctypes.c_uint64, ctypes.c_int]
        L.orc_phi4_step_slab.argtypes = [ctypes.POINTER(Phi4), _F, _F, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_uint64]
        L.orc_phi4_init.argtypes = [ctypes.POINTER(Phi4), ctypes.c_float, _F]
        L.orc_phi4_step_stab.argtypes = [ctypes.POINTER(Phi4), _F, _F, ctypes.c_uint64, _F]
        L.orc_phi4_stab_rule.restype = ctypes.c_int
        L.orc_phi4_stab_rule.argtypes = [_F, _F, _F, _F, _F, ctypes.c_int]
        L.orc_phi4_step_range.argtypes = [ctypes.POINTER(Phi4), _F, _F, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_phi4_sigma.restype = ctypes.c_float
        L.orc_phi4_sigma.argtypes = [ctypes.c_float, ctypes.c_double]
        _lib = L
    return _lib


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def normals(seed, stream, quad0, step, nquads):
    out = np.empty(4 * nquads, dtype=np.float32)
    L = lib()
    tmp = (ctypes.c_float * 4)()
    for q in range(nquads):
        L.orc_normals4(seed, stream, quad0 + q, step, tmp)
        out[4 * q:4 * q + 4] = tmp[:]
    return out


def qm1d_frame(N, a, dtau, pot, C, loops, seed, tick, runs, f, x, xx0, omega, lrgEl=0, lrgVl=0.0):
    """One Jacobi-semantics frame (the GPU's contract); returns a dict."""
    f = np.ascontiguousarray(f, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    xx0 = np.ascontiguousarray(xx0, dtype=np.float64)
    nf, nx, nxx0 = np.empty(N), np.empty(N), np.empty(N)
    s = Qm1d(N=N, pot=pot, loops=loops, a=a, c=C, dtau=dtau, seed=seed, tick=tick, runs=runs,
             f=f.ctypes.data_as(_D), x=x.ctypes.data_as(_D), xx0=xx0.ctypes.data_as(_D),
             nf=nf.ctypes.data_as(_D), nx=nx.ctypes.data_as(_D), nxx0=nxx0.ctypes.data_as(_D),
             omega=omega, lrgEl=lrgEl, lrgVl=lrgVl)
    lib().orc_qm1d_frame(ctypes.byref(s))
    return {"f": nf, "x": nx, "xx0": nxx0, "omega": s.nomega, "lrgEl": s.lrgEl, "lrgVl": s.lrgVl,
            "stable": s.stable, "steps_done": s.steps_done}


_BM_TABLES = None


class device_transcendentals:
    """Context manager: the oracle's normals use the device's Box-Muller
    factors (sq_selftest_bm_tables, 4 x 2^23 float32), so its noise -- and with
    it every noise-on result -- is the GPU's bit for bit."""

    def __init__(self, tables):
        self.tables = np.ascontiguousarray(tables, dtype=np.float32)
        assert self.tables.size == 4 << 23

    def __enter__(self):
        global _BM_TABLES
        _BM_TABLES = self.tables  # keep the buffer alive while the C side points at it
        lib().orc_set_bm_tables(self.tables.ctypes.data_as(_F))
        return self

    def __exit__(self, *exc):
        global _BM_TABLES
        lib().orc_set_bm_tables(None)
        _BM_TABLES = None
        return False


def libm_f32(fn, x):
    """The host libm's logf (fn 0), cosf (1) or tanhf (2) of a float32 array."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    lib().orc_libm_f32(fn, x.ctypes.data_as(_F), y.ctypes.data_as(_F), x.size)
    return y


def ref_noise_stream(seed, N, loops):
    """The reference's random() draws of one full launch in call order
    (k = round*(N+1) + item): xi, the accepted draws' words t1>>16 and t2>>16,
    and the shared seed after each call."""
    n = (N + 1) * loops
    xi = np.empty(n)
    w1 = np.empty(n, dtype=np.uint32)
    w2 = np.empty(n, dtype=np.uint32)
    seeds = np.empty(n, dtype=np.uint64)
    lib().orc_ref_noise_stream(seed, N, loops, xi.ctypes.data_as(_D), w1.ctypes.data_as(_U32),
                               w2.ctypes.data_as(_U32), seeds.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    return xi, w1, w2, seeds


class SerialChain:
    """The reference's device state under the serial semantics, frame by frame
    (orc_serial_launch = one clEnqueueNDRangeKernel of time_dev), with the
    host loop of tauhost.c:504-554: stable -> adopt new*, runs += loops;
    either way re-upload f, x, xx0, omega.  newf, lrgEl, lrgVl and the seed
    are never rolled back (tauhost.c)."""

    def __init__(self, N, a, dtau, pot, C, loops, seed, f, x=None, xx0=None, omega=0.0, runs=0, adapt=True):
        self.N = N
        self.adapt = adapt
        self.stab_cnt = 0
        self.host = {"f": np.array(f, dtype=np.float64), "x": np.zeros(N) if x is None else np.array(x, float),
                     "xx0": np.zeros(N) if xx0 is None else np.array(xx0, float)}
        self.buf = {k: np.array(self.host[k]) for k in ("f", "x", "xx0")}
        self.buf.update({"nf": np.array(self.host["f"]), "nx": np.array(self.host["x"]),
                         "nxx0": np.array(self.host["xx0"])})
        self.d = SerialDev(N=N, pot=pot, loops=loops, a=a, c=C, omega=omega, seed=seed, stable=1,
                           dtau=dtau, lrgEl=0, lrgVl=0.0, runs=runs)
        for k, v in self.buf.items():
            setattr(self.d, k, v.ctypes.data_as(_D))
        self.omega = omega
        self.runs = runs

    def frame(self):
        d = self.d
        lib().orc_serial_launch(ctypes.byref(d))
        stable = d.stable
        if stable == 1:
            for k in ("f", "x", "xx0"):
                self.host[k][:] = self.buf["n" + k]
            self.omega = d.omega
            if self.adapt:                        # tauhost.c:523-528
                if self.stab_cnt > 10:
                    self.stab_cnt = 0
                    d.dtau = d.dtau / 0.950
                self.stab_cnt += 1
            self.runs += d.loops
        elif self.adapt:                          # :537-541
            d.dtau = d.dtau * 0.950
            self.stab_cnt = 0
        d.stable = 1
        for k in ("f", "x", "xx0"):
            self.buf[k][:] = self.host[k]
        d.omega = self.omega
        d.runs = self.runs
        return stable


def phi4_params(shape, h, m2, lam, seed, clamp=1000.0, C=1.0):
    Lx, Ly, Lz = shape
    return Phi4(Lx=Lx, Ly=Ly, Lz=Lz, h=h, m2=m2, lam=lam, clampv=clamp, seed=seed, C=C)


def phi4_step(p, phi, step, nthreads=0):
    a = np.ascontiguousarray(phi, dtype=np.float32)
    out = np.empty_like(a)
    lib().orc_phi4_step(ctypes.byref(p), a.ctypes.data_as(_F), out.ctypes.data_as(_F), step, nthreads)
    return out


def phi4_step_slab(p, padded, z0, step):
    """padded: (nz+2, Ly, Lx) with ghost planes; returns the nz updated planes."""
    a = np.ascontiguousarray(padded, dtype=np.float32)
    nz = a.shape[0] - 2
    out = np.empty((nz,) + a.shape[1:], dtype=np.float32)
    lib().orc_phi4_step_slab(ctypes.byref(p), a.ctypes.data_as(_F), out.ctypes.data_as(_F), nz, z0, step)
    return out


def phi4_step_range(p, src, dst, gpad, lo, hi, z0, step):
    """Update planes [lo, hi) (local, may reach into the ghost zones) of the
    padded slab `dst` ((nz + 2 gpad, Ly, Lx) float32, modified in place) from
    the padded slab `src`; global z wraps modulo Lz."""
    assert src.dtype == np.float32 and dst.dtype == np.float32 and src.flags.c_contiguous and dst.flags.c_contiguous
    nz = src.shape[0] - 2 * gpad
    assert -gpad < lo and hi < nz + gpad, "the range needs one readable plane on either side"
    lib().orc_phi4_step_range(ctypes.byref(p), src.ctypes.data_as(_F), dst.ctypes.data_as(_F), nz, gpad, lo, hi,
                              z0, step)


def phi4_frame_stab(p, phi, steps, step0, T, V):
    """`steps` steps from phi with the per-step stability records and the
    frame rule: returns (phi', M, D, A, fired, T', V')."""
    phi = np.ascontiguousarray(phi, dtype=np.float32)
    M, D, A = (np.zeros(steps, np.float32) for _ in range(3))
    rec = np.zeros(3, np.float32)
    for j in range(steps):
        out = np.empty_like(phi)
        lib().orc_phi4_step_stab(ctypes.byref(p), phi.ctypes.data_as(_F), out.ctypes.data_as(_F), step0 + j,
                                 rec.ctypes.data_as(_F))
        M[j], D[j], A[j] = rec
        phi = out
    t = np.array([T], np.float32)
    v = np.array([V], np.float32)
    fired = lib().orc_phi4_stab_rule(t.ctypes.data_as(_F), v.ctypes.data_as(_F), M.ctypes.data_as(_F),
                                     D.ctypes.data_as(_F), A.ctypes.data_as(_F), steps)
    return phi, M, D, A, fired, float(t[0]), float(v[0])


def phi4_init(p, amp):
    out = np.empty((p.Lz, p.Ly, p.Lx), dtype=np.float32)
    lib().orc_phi4_init(ctypes.byref(p), amp, out.ctypes.data_as(_F))
    return out


def tauhost(argv, cwd):
    """Run the serial-reference-semantics CLI (orc_tauhost) with tauhost.c's argv."""
    if not os.path.exists(CLI):
        build()
    return subprocess.run([CLI] + [str(a) for a in argv], cwd=cwd, capture_output=True, timeout=300)
