"""stochquant_amd -- MI355X-native (gfx950) drop-in for SebTanz/StochQuant's
stochastic-quantisation Langevin path.

    libstochquant.so   HIP kernels + C ABI (include/stochquant.h)
    tauhost.o          the reference's CLI executable over that ABI
    langevin           numpy-level mirror used by tests and bench.py

The package imports without a GPU; every compute call goes through the HIP
library and raises if it is unavailable (there is no CPU fallback).
"""
from ._lib import (LIB_PATH, TAUHOST_PATH, StochQuantError, StochQuantUnavailable, device_count,
                   load)
from .langevin import (Phi4Lattice, Qm1dChain, connect_p2p, parse_frame_line, run_tauhost, tauhost_argv,
                       unique_id)

__all__ = [
    "LIB_PATH", "TAUHOST_PATH", "StochQuantError", "StochQuantUnavailable", "device_count", "load",
    "Phi4Lattice", "Qm1dChain", "connect_p2p", "parse_frame_line", "run_tauhost", "tauhost_argv", "unique_id",
]
