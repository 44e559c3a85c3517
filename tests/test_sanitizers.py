"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only;
GPU sanitizers are not available on the pool).

  * the serial oracle (oracle/, the reference's semantics incl. its start-file
    parser) on the recorded reference runs, fresh and resumed;
  * the drop-in tauhost.o's own host code (argv handling, start-file parser,
    error paths) up to the point where it needs a GPU.
"""
import os
import shutil
import subprocess

import pytest

from conftest import golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _gxx_has_asan():
    r = subprocess.run(["gcc", "-fsanitize=address", "-x", "c", "-", "-o", os.devnull],
                       input=b"int main(void){return 0;}", capture_output=True)
    return r.returncode == 0


pytestmark = pytest.mark.skipif(not _gxx_has_asan(), reason="gcc without ASan runtime")


@pytest.fixture(scope="module")
def san_oracle():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(ROOT, "oracle", "_san", "orc_tauhost_san")


def _run(exe, argv, cwd):
    a = ["end" if v == "END" else ("start" if v == "START" else v) for v in argv]
    return subprocess.run([exe] + a, cwd=cwd, capture_output=True, env=ENV, timeout=600)


def test_oracle_reference_runs_clean(san_oracle, tmp_path):
    g = golden("reference_outputs.json")
    r = _run(san_oracle, g["appendix_c_end_file"]["argv"], tmp_path)
    assert r.returncode == 0, r.stderr.decode()
    assert (tmp_path / "end").read_text().split("\n")[0] == g["appendix_c_end_file"]["first_line"]
    r = _run(san_oracle, g["double_well_stable"]["argv"], tmp_path)
    assert r.returncode == 0, r.stderr.decode()
    shutil.copy(tmp_path / "end", tmp_path / "start")
    r = _run(san_oracle, g["resume_double_count"]["resume_argv"], tmp_path)
    assert r.returncode == 0, r.stderr.decode()
    assert b"ERROR: AddressSanitizer" not in r.stderr and b"runtime error" not in r.stderr


def test_oracle_malformed_start_file(san_oracle, tmp_path):
    """Short lines, missing fields and no trailing newline: the parser must
    not read out of bounds (tauhost.c:119-146 runs strtok on such lines)."""
    (tmp_path / "start").write_bytes(b"0x1p-3|0x1p-4\n|||\n\n0.5\n12|N\n0.01|deltaTau")
    r = _run(san_oracle, ["4", "0.5", "0.01", "1", "0", "1", "0", "1", "0", "5", "START", "0", "12"], tmp_path)
    assert b"ERROR: AddressSanitizer" not in r.stderr and b"runtime error" not in r.stderr, r.stderr.decode()


@pytest.fixture(scope="module")
def san_tauhost(tmp_path_factory):
    """tauhost.cpp built with the sanitizers against the real libstochquant.so."""
    out = str(tmp_path_factory.mktemp("san") / "tauhost_san")
    lib = os.path.join(ROOT, "stochquant_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libstochquant.so")):
        pytest.skip("libstochquant.so not built")
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-o", out,
                        os.path.join(ROOT, "stochquant_amd", "csrc", "tauhost.cpp"), f"-L{lib}", "-lstochquant",
                        f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib", "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


@pytest.mark.parametrize("start", [b"", b"0.1|0.2|0.3|0.4\n", b"a|b\n|\n\n\n\n\n\n\n",
                                   b"0x1p-3| 0x1p-4| 0x1p-5| 0x1p-6\n" * 4 + b"0|omega\n7|N\n0.5|deltaTau\n"])
def test_tauhost_host_code_clean(san_tauhost, tmp_path, start):
    """Parses the start file and stops at 'no HIP device' (no GPU here) or runs
    (GPU present): either way no sanitizer report."""
    (tmp_path / "start").write_bytes(start)
    r = _run(san_tauhost, ["4", "0.5", "0.01", "1", "0", "1", "0", "1", "0", "5", "START", "0", "12"], tmp_path)
    assert b"ERROR: AddressSanitizer" not in r.stderr and b"runtime error" not in r.stderr, r.stderr.decode()
    assert r.returncode in (0, 1)
    r = _run(san_tauhost, ["4", "0.5"], tmp_path)          # too few arguments
    assert r.returncode == 1 and b"runtime error" not in r.stderr
