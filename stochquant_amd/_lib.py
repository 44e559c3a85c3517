"""ctypes binding of libstochquant.so (include/stochquant.h).

The library is the product: there is no Python or CPU fallback.  If the
shared object is missing or cannot be loaded, `load()` raises
`StochQuantUnavailable` -- callers must not silently route elsewhere.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "lib", "libstochquant.so")
TAUHOST_PATH = os.path.join(_PKG, "bin", "tauhost.o")

SQ_OK = 0
SQ_MODEL_QM1D = 0
SQ_MODEL_PHI4 = 1
SQ_COMM_NONE = 0
SQ_COMM_LOOPBACK = 1
SQ_COMM_RCCL = 2
SQ_COMM_P2P = 3
SQ_P2P_HANDLE_BYTES = 512
SQ_ORDER_JACOBI = 0
SQ_ORDER_SERIAL = 1


class StochQuantUnavailable(RuntimeError):
    """libstochquant.so is missing or unloadable (build it: python -m stochquant_amd.build)."""


class StochQuantError(RuntimeError):
    """A libstochquant call returned a negative status."""

    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


class SqParams(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_int),
        ("model", ctypes.c_int),
        ("dims", ctypes.c_longlong * 3),
        ("deltat", ctypes.c_double),
        ("deltatau", ctypes.c_double),
        ("pot", ctypes.c_int),
        ("C", ctypes.c_double),
        ("loops", ctypes.c_int),
        ("seed", ctypes.c_ulonglong),
        ("m2", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("clamp", ctypes.c_double),
        ("device", ctypes.c_int),
        ("adapt_dtau", ctypes.c_int),
        ("comm", ctypes.c_int),
        ("nranks", ctypes.c_int),
        ("rank", ctypes.c_int),
        ("nslabs", ctypes.c_int),
        ("comm_id", ctypes.c_ubyte * 128),
    ]


class SqPerf(ctypes.Structure):
    _fields_ = [
        ("steps", ctypes.c_longlong),
        ("site_updates", ctypes.c_longlong),
        ("step_kernel_ms", ctypes.c_double),
        ("step_kernel_launches", ctypes.c_longlong),
        ("frame_ms", ctypes.c_double),
        ("halo_bytes", ctypes.c_double),
        ("kernel_launches", ctypes.c_longlong),
        ("fused_steps", ctypes.c_longlong),
    ]


class SqBlockOp(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("step", ctypes.c_int), ("lo", ctypes.c_int), ("hi", ctypes.c_int),
                ("lo2", ctypes.c_int), ("hi2", ctypes.c_int), ("stream", ctypes.c_int)]


(SQ_OP_EXCHANGE, SQ_OP_STEP, SQ_OP_PAIR, SQ_OP_WAIT_EXCHANGE, SQ_OP_EDGES_DONE, SQ_OP_WAIT_STAGED, SQ_OP_SIGNAL,
 SQ_OP_WAIT) = range(8)
ABI_VERSION = 6


_P = ctypes.c_void_p
_D = ctypes.POINTER(ctypes.c_double)
_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes); every symbol here is declared in include/stochquant.h
SIGNATURES = {
    "sq_params_init": (None, [ctypes.POINTER(SqParams)]),
    "sq_last_error": (ctypes.c_char_p, []),
    "sq_abi_version": (ctypes.c_int, []),
    "sq_create": (ctypes.c_int, [ctypes.POINTER(SqParams), ctypes.POINTER(_P)]),
    "sq_destroy": (ctypes.c_int, [_P]),
    "sq_upload": (ctypes.c_int, [_P, _D, _D, _D, ctypes.c_double, ctypes.c_long]),
    "sq_download": (ctypes.c_int, [_P, _D, _D, _D, _D, ctypes.POINTER(ctypes.c_long)]),
    "sq_qm1d_get_scan": (ctypes.c_int, [_P, _I, _D, ctypes.POINTER(ctypes.c_ulonglong)]),
    "sq_qm1d_set_scan": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_double, ctypes.c_ulonglong]),
    "sq_run_frame": (ctypes.c_int, [_P, _I]),
    "sq_run_frames": (ctypes.c_int, [_P, ctypes.c_int, _I, _D]),
    "sq_step": (ctypes.c_int, [_P, ctypes.c_int]),
    "sq_upload_field": (ctypes.c_int, [_P, _F, ctypes.c_size_t]),
    "sq_download_field": (ctypes.c_int, [_P, _F, ctypes.c_size_t]),
    "sq_init_field": (ctypes.c_int, [_P, ctypes.c_float]),
    "sq_init_field_hash": (ctypes.c_int, [_P, ctypes.c_double, ctypes.c_ulonglong]),
    "sq_slab": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]),
    "sq_moments": (ctypes.c_int, [_P, _D]),
    "sq_phi4_tile": (ctypes.c_int, [_P, _I]),
    "sq_get_params": (ctypes.c_int, [_P, ctypes.POINTER(SqParams)]),
    "sq_save_field": (ctypes.c_int, [_P, ctypes.c_char_p]),
    "sq_load_field": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int]),
    "sq_phi4_kernel": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t]),
    "sq_phi4_ghost": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "sq_phi4_schedule": (ctypes.c_int, [_P, _I, _I, _I]),
    "sq_phi4_edge_first": (ctypes.c_int, [_P, _I]),
    "sq_phi4_exchange_stream": (ctypes.c_int, [_P, _I, _I]),
    "sq_phi4_block_plan": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.POINTER(SqBlockOp), ctypes.c_int, _I]),
    "sq_phi4_pick_ghost": (ctypes.c_int, [_D, ctypes.c_int]),
    "sq_phi4_stability": (ctypes.c_int, [_P, _D, _I, _F, _F, _F, ctypes.c_int]),
    "sq_phi4_set_stability": (ctypes.c_int, [_P, ctypes.c_double, ctypes.c_double]),
    "sq_qm1d_set_ordering": (ctypes.c_int, [_P, ctypes.c_int]),
    "sq_qm1d_set_lcg_seed": (ctypes.c_int, [_P, ctypes.c_ulonglong]),
    "sq_qm1d_get_lcg_seed": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ulonglong)]),
    "sq_qm1d_inject_noise": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t]),
    "sq_qm1d_noise_consumed": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ulonglong)]),
    "sq_selftest_lcg": (ctypes.c_int, [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint),
                                       ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_double),
                                       ctypes.c_int]),
    "sq_set_dtau": (ctypes.c_int, [_P, ctypes.c_double]),
    "sq_get_dtau": (ctypes.c_int, [_P, _D]),
    "sq_get_step": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ulonglong)]),
    "sq_set_step": (ctypes.c_int, [_P, ctypes.c_ulonglong]),
    "sq_correlator": (ctypes.c_int, [_P, _D, ctypes.c_int]),
    "sq_set_profiling": (ctypes.c_int, [_P, ctypes.c_int]),
    "sq_perf": (ctypes.c_int, [_P, ctypes.POINTER(SqPerf)]),
    "sq_perf_reset": (ctypes.c_int, [_P]),
    "sq_sync": (ctypes.c_int, [_P]),
    "sq_phi4_launch_info": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_longlong),
                                           ctypes.POINTER(ctypes.c_longlong)]),
    "sq_build_id": (ctypes.c_char_p, []),
    "sq_set_noise": (ctypes.c_int, [_P, ctypes.c_double]),
    "sq_phi4_block_stamps": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, _I]),
    "sq_phi4_block_clocks": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, _I]),
    "sq_comm_unique_id": (ctypes.c_int, [ctypes.POINTER(ctypes.c_ubyte)]),
    "sq_p2p_handle": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ubyte)]),
    "sq_p2p_connect": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_ubyte), ctypes.c_int]),
    "sq_device_count": (ctypes.c_int, [_I]),
    "sq_selftest_normals": (ctypes.c_int, [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_uint,
                                           ctypes.c_ulonglong, ctypes.c_ulonglong, _F, ctypes.c_size_t]),
    "sq_selftest_dpp": (ctypes.c_int, [ctypes.c_int, _F]),
    "sq_selftest_dpp_mix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_uint)]),
    "sq_selftest_philox": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint), ctypes.POINTER(ctypes.c_uint),
                                          ctypes.POINTER(ctypes.c_uint)]),
    "sq_copy_bandwidth": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, _D]),
    "sq_selftest_libm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _F, _F, ctypes.c_longlong]),
    "sq_selftest_bm_tables": (ctypes.c_int, [ctypes.c_int, _F]),
}

_lib = None


def load(path=None):
    """Load libstochquant.so once; raise StochQuantUnavailable if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("SQ_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise StochQuantUnavailable(f"{p} not found; build it with `python -m stochquant_amd.build`")
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise StochQuantUnavailable(f"cannot load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sq_abi_version() != ABI_VERSION:
        raise StochQuantUnavailable("ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(fn_name, rc):
    if rc != SQ_OK:
        msg = load().sq_last_error()
        raise StochQuantError(fn_name, rc, msg.decode() if msg else "")
    return rc


def call(fn_name, *args):
    return check(fn_name, getattr(load(), fn_name)(*args))


def default_params():
    p = SqParams()
    load().sq_params_init(ctypes.byref(p))
    return p


def build_id():
    """{"phi4": <hash of the φ⁴ kernels' code object>, "lib": <hash of every object>} of the loaded library."""
    s = load().sq_build_id().decode()
    return dict(kv.split(":", 1) for kv in s.split() if ":" in kv) or {"raw": s}


def device_count():
    n = ctypes.c_int(0)
    call("sq_device_count", ctypes.byref(n))
    return n.value
