"""The drop-in boundary without a GPU: libstochquant.so loads, exports every
symbol include/stochquant.h declares, its struct layout matches the binding,
compute entry points fail loudly (no CPU fallback), and tauhost.o keeps the
reference's CLI error behaviour (tauhost.c:105-107)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "stochquant.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sq_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(sqlib):
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(sqlib, s)]
    assert missing == []


def test_binding_covers_header():
    from stochquant_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_params_layout_and_defaults(sqlib):
    from stochquant_amd import _lib
    p = _lib.default_params()
    assert p.struct_size == ctypes.sizeof(_lib.SqParams)
    assert p.clamp == 1000.0          # tau_kernel.cl:61
    assert p.adapt_dtau == 1          # tauhost.c:523-541
    assert sqlib.sq_abi_version() == _lib.ABI_VERSION == 6


def test_no_silent_cpu_fallback(sqlib):
    """Without a device, sq_create returns SQ_E_NODEV and the Python layer raises."""
    from stochquant_amd import _lib, Qm1dChain, StochQuantError
    if _lib.device_count() > 0:
        pytest.skip("GPU present: covered by the gpu tests")
    with pytest.raises(StochQuantError) as ei:
        Qm1dChain(16, 0.1, 0.002)
    assert ei.value.code == -5


def test_library_is_gfx950_code_object(sqlib):
    """The fat binary embedded in the library carries a gfx950 code object."""
    from stochquant_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"phi4_step_kernel" in blob


def test_tauhost_cli_errors_without_gpu(sqlib, tmp_path):
    from stochquant_amd import _lib
    exe = _lib.TAUHOST_PATH
    r = subprocess.run([exe], capture_output=True, cwd=tmp_path)
    assert r.returncode == 1
    r = subprocess.run([exe, "4", "0.5", "0.01", "1", "0", "1", "0", "1", "0", "5", "missing", "0", "12"],
                       capture_output=True, cwd=tmp_path)
    assert r.returncode == 1
    assert b"Failed to read Input." in r.stderr


def test_taumain_argv_contract():
    """taumain.py:132 builds 13 string arguments in this order."""
    from stochquant_amd import tauhost_argv, TAUHOST_PATH
    a = tauhost_argv(200, 0.02, 0.002, 5000, 3, 1.0, 2, 1, 0, 1000, "0", "V0_2e_0-8.txt", 40)
    assert a[0] == TAUHOST_PATH
    assert a[1:] == ["200", "0.02", "0.002", "5000", "3", "1.0", "2", "1", "0", "1000", "0",
                     "V0_2e_0-8.txt", "40"]


def test_frame_line_parser_matches_taumain():
    from stochquant_amd import parse_frame_line
    r = parse_frame_line(b" -inf | -inf | -inf | 0.01000000000000000021 |  50.00\n")
    assert list(r["y"]) == [float("-inf")] * 3
    assert r["dtau"] == 0.01 and r["percent"] == 50.0


def test_driver_presets_mirror_taumain():
    """stochquant_amd.driver.PRESETS / preset_argv = taumain.py:91-132."""
    from stochquant_amd.driver import PRESETS, preset_argv
    assert PRESETS["double_well"] == {"dtau": .002, "Nt": 200, "dt": .02, "potID": 3, "theoVal": 10, "c": 1.,
                                      "filename": "V0_2e_0-8.txt"}
    assert PRESETS["harmosc"]["dtau"] == .3 and PRESETS["harmosc"]["Nt"] == 100
    argv = preset_argv("double_well", exe="./tauhost.o")
    assert argv == ["./tauhost.o", "200", "0.02", "0.002", "5000", "3", "1.0", "2", "1", "0", "1000", "0",
                    "V0_2e_0-8.txt", "40"]
