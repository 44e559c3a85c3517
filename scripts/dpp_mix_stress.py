"""Cross-wave DPP stress (sq_selftest_dpp_mix): counts of wrong wave_ror/rol
results per lane for each mode, printed as one JSON line per mode."""
import ctypes
import json
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stochquant_amd import _lib  # noqa: E402

lib = _lib.load()
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 512
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
for mode in (0, 1, 2, 3):
    for rep in range(2):
        e = np.zeros(64, dtype=np.uint32)
        rc = lib.sq_selftest_dpp_mix(0, mode, blocks, iters, e.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)))
        assert rc == 0, _lib.load().sq_last_error()
        bad = [int(i) for i in np.nonzero(e)[0]]
        print(json.dumps({"mode": mode, "rep": rep, "blocks": blocks, "iters": iters, "wrong": int(e.sum()),
                          "lanes": bad[:64]}), flush=True)
