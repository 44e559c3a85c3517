"""tauhost.o (the drop-in executable) end to end on the MI355X, against the
reference's recorded outputs (tests/golden/reference_outputs.json).

By default (N <= 4096) tauhost.o runs the reference's own serial order with
its LCG seeded from the same rand() draw and glibc's float log/cos/tanh
algorithms on the device (csrc/sq_glibcf.h), so its stdout and end file are
the serial oracle's byte for byte and the recorded reference values bit for
bit: formats, initial state (same unseeded glibc rand() draws,
tauhost.c:84-102), first printed frame (xavg = 0 -> all -inf), trajectory, Δτ
controller sequence, omega and trailer lines.  SQ_ORDER=jacobi (and N > 4096) runs the
Jacobi / Philox frame, checked statistically against its own exact law.
"""
import re
import shutil

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

HEX = r"-?0x[0-9a-f]+(\.[0-9a-f]+)?p[-+]\d+"


def _run(tmp_path, argv):
    from stochquant_amd import TAUHOST_PATH, run_tauhost
    a = ["end" if v == "END" else ("start" if v == "START" else v) for v in argv]
    r = run_tauhost([TAUHOST_PATH] + list(a), cwd=str(tmp_path), timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    end = (tmp_path / "end").read_text() if (tmp_path / "end").exists() else None
    return r.stdout.decode(), end


def test_appendix_c_run_jacobi(gpu, tmp_path):
    g = golden("reference_outputs.json")["appendix_c_end_file"]
    out, end = _run_env(tmp_path, g["argv"], SQ_ORDER="jacobi")
    lines = out.split("\n")
    assert lines[0] == g["stdout_first_line"]
    assert re.fullmatch(r"( -?\d+\.\d{20} \|){3} 0\.01000000000000000021 \|  100\.00", lines[1])
    el = end.split("\n")
    assert el[4:7] == g["trailer"]          # omega bit-exact (potID 0), N, deltaTau
    for ln in el[:4]:
        f = [t.strip() for t in ln.split("|")]
        assert len(f) == 4 and all(re.fullmatch(HEX, t) for t in f)


def test_all_unstable_preset_dtau_sequence_jacobi(gpu, tmp_path):
    g = golden("reference_outputs.json")["double_well_all_unstable"]
    out, end = _run_env(tmp_path, g["argv"], SQ_ORDER="jacobi")
    dt = [ln.split("|")[-2].strip() for ln in out.strip().split("\n")]
    assert dt == g["printed_dtau"]
    tail = end.strip().split("\n")[-3:]
    assert float(tail[2].split("|")[0]) == pytest.approx(g["end_dtau"], rel=1e-6)
    assert int(tail[1].split("|")[0]) == g["end_N"]


def test_stable_preset_and_resume(gpu, tmp_path):
    from stochquant_amd import parse_frame_line
    g = golden("reference_outputs.json")
    out, end = _run(tmp_path, g["double_well_stable"]["argv"])
    assert int(end.strip().split("\n")[-2].split("|")[0]) == g["double_well_stable"]["end_N"]
    for ln in out.strip().split("\n"):
        r = parse_frame_line(ln.encode())
        assert r["y"].size == 199 and r["dtau"] == pytest.approx(0.002)
    shutil.copy(tmp_path / "end", tmp_path / "start")
    _, end2 = _run(tmp_path, g["resume_double_count"]["resume_argv"])
    assert int(end2.strip().split("\n")[-2].split("|")[0]) == g["resume_double_count"]["resume_end_N"]


@pytest.mark.parametrize("order", ["serial", "jacobi"])
def test_plotted_correlator_matches_exact_stationary_value(gpu, tmp_path, order):
    """The curve taumain.py plots, log|xavg| (xavg = running <X_i X_mid> -
    <X_i><X_mid>, tauhost.c:519-521), from a 60-frame tauhost.o run converges
    to the exact stationary connected correlator of the chain's ordering
    (tests/qm1d_exact.py): the default serial order (the reference's
    Gauss-Seidel sweep) and SQ_ORDER=jacobi have different O(dtau) stationary
    laws, so each run is compared with its own exact law.  ~150 independent
    samples -> 2.5 sigma = 30 %."""
    from qm1d_exact import stationary_cov
    from stochquant_amd import parse_frame_line
    argv = ["100", "0.1", "0.002", "60", "0", "1", "0", "1", "0", "1000", "0", "end", "17"]
    out_gpu, _ = _run_env(tmp_path, argv, SQ_ORDER=order)
    y = parse_frame_line(out_gpu.strip().split("\n")[-1].encode())["y"]   # sites 1..N-1
    c = np.exp(y[39:59])                                                    # sites 40..59
    exact = stationary_cov(100, 0.1, 0.002, "jacobi" if order == "jacobi" else "gs")[40:60, 50]
    assert np.all(np.isfinite(c))
    assert abs(c.mean() - exact.mean()) < 0.3 * exact.mean()


def test_config_c1_chain_through_tauhost(gpu, tmp_path):
    """BASELINE configs[0] / SURVEY §8d C1: the "32^3" chain = N = 32,768 sites,
    dt = 1, dtau = 0.01, potID 0, C = 1, 1000 steps, fresh start, via the
    drop-in executable.  The bulk <f^2> relaxes to the exact Euler-Maruyama
    value 0.29378 (tests/golden/analytic_kats.json; the survey's serial oracle
    run gave 0.2943)."""
    g = golden("analytic_kats.json")["free_var_1d"]
    argv = ["32768", "1.0", "0.01", "1", "0", "1", "0", "1", "0", "1000", "0", "END", "17"]
    out, end = _run(tmp_path, argv)
    lines = end.strip().split("\n")
    f = np.array([float.fromhex(ln.split("|")[3].strip()) for ln in lines[:32768]])
    bulk = f[256:-256]
    m2 = np.mean(bulk ** 2)
    err = 2 * np.std(bulk ** 2) / np.sqrt(bulk.size) * 3   # ~3 sites correlation length
    assert abs(m2 - g["value"]) < 4 * err
    assert lines[-2].strip() == "1000|N"


def _run_env(tmp_path, argv, **env):
    import os
    from stochquant_amd import TAUHOST_PATH, run_tauhost
    a = ["end" if v == "END" else ("start" if v == "START" else v) for v in argv]
    e = dict(os.environ)
    e.update(env)
    r = run_tauhost([TAUHOST_PATH] + list(a), cwd=str(tmp_path), timeout=300, env=e)
    assert r.returncode == 0, r.stderr.decode()
    if env.get("SQ_MODEL") == "phi4":   # binary checkpoint: the caller np.load()s it
        return r.stdout.decode(), None
    return r.stdout.decode(), (tmp_path / "end").read_text()


def _hexrows(text, n):
    return np.array([[float.fromhex(t.strip()) for t in ln.split("|")] for ln in text.split("\n")[:n]])


def test_serial_order_reproduces_appendix_c(gpu, oracle_mod, tmp_path):
    """Default order (no SQ_ORDER): the reference's serial order with its LCG
    seeded from the same rand() draw and glibc's float log/cos on the device:
    the recorded end-file line, the serial oracle's
    whole end file, stdout, omega, N and deltaTau, all bit for bit."""
    g = golden("reference_outputs.json")["appendix_c_end_file"]
    out, end = _run(tmp_path, g["argv"])
    assert out.split("\n")[0] == g["stdout_first_line"]
    el = end.split("\n")
    assert el[4:7] == g["trailer"]
    got = _hexrows(end, 4)
    first = np.array([float.fromhex(t.strip()) for t in g["first_line"].split("|")])
    assert np.array_equal(got[0], first), (got[0], first)
    ref_dir = tmp_path / "orc"
    ref_dir.mkdir()
    a = ["end" if v == "END" else v for v in g["argv"]]
    r = oracle_mod.tauhost(a, cwd=str(ref_dir))
    assert r.returncode == 0
    ref = _hexrows((ref_dir / "end").read_text(), 4)
    assert np.array_equal(got, ref), (got, ref)
    assert end == (ref_dir / "end").read_text()


@pytest.mark.parametrize("case", ["appendix_c_end_file", "double_well_all_unstable", "double_well_stable"])
def test_reference_runs_byte_identical_to_oracle(gpu, oracle_mod, tmp_path, case):
    """The recorded reference runs (potID 0 and the double-well presets, potID
    3): tauhost.o's stdout and end file equal the serial oracle's byte for byte."""
    g = golden("reference_outputs.json")[case]
    out, end = _run(tmp_path, g["argv"])
    ref_dir = tmp_path / "orc"
    ref_dir.mkdir()
    a = ["end" if v == "END" else v for v in g["argv"]]
    r = oracle_mod.tauhost(a, cwd=str(ref_dir))
    assert r.returncode == 0
    assert out == r.stdout.decode()
    assert end == (ref_dir / "end").read_text()


def test_serial_order_all_unstable_preset(gpu, tmp_path):
    """The double-well all-unstable preset in the default (serial) order: same
    printed Δτ sequence and end Δτ / N as the reference's recorded run."""
    g = golden("reference_outputs.json")["double_well_all_unstable"]
    out, end = _run(tmp_path, g["argv"])
    dt = [ln.split("|")[-2].strip() for ln in out.strip().split("\n")]
    assert dt == g["printed_dtau"]
    tail = end.strip().split("\n")[-3:]
    assert float(tail[2].split("|")[0]) == pytest.approx(g["end_dtau"], rel=1e-6)
    assert int(tail[1].split("|")[0]) == g["end_N"]


def test_phi4_mode_through_the_cli(gpu, tmp_path):
    """SQ_MODEL=phi4: the 3-D lattice behind the reference's 13 arguments.
    stdout is taumain-parseable (Lz-1 values, dtau, percent; first frame -inf
    like the reference's), the end file is a binary checkpoint, a START resume
    continues the noise stream bit for bit, and the field equals the library
    run with the same seed."""
    from stochquant_amd import Phi4Lattice, parse_frame_line
    env = dict(SQ_MODEL="phi4", SQ_SHAPE="64x16x32", SQ_SEED="7", SQ_M2="0.5", SQ_LAMBDA="1.5")
    argv = lambda frames, start: ["32", "1", "0.01", str(frames), "0", "1", "0", "1", "0", "10", start, "END", "12"]
    out, _ = _run_env(tmp_path, argv(4, "0"), SQ_PERF_JSON=str(tmp_path / "perf.json"), **env)
    import json
    perf = json.loads((tmp_path / "perf.json").read_text())
    assert perf["model"] == "phi4" and perf["steps"] == 40 and perf["site_updates"] == 40 * 64 * 16 * 32
    lines = out.strip().split("\n")
    assert len(lines) == 4
    for k, ln in enumerate(lines):
        r = parse_frame_line(ln.encode())
        assert r["y"].size == 31 and r["dtau"] == pytest.approx(0.01) and r["percent"] == pytest.approx(25 * (k + 1))
    assert np.all(np.isneginf(parse_frame_line(lines[0].encode())["y"]))
    assert np.all(np.isfinite(parse_frame_line(lines[-1].encode())["y"]))
    full = np.load(tmp_path / "end")
    import json
    meta = json.loads((tmp_path / "end.json").read_text())
    assert full.shape == (32, 16, 64) and meta["step"] == 40 and meta["dims"] == [64, 16, 32]
    # resume: 2 frames, then 2 more from the checkpoint
    d2 = tmp_path / "r"
    d2.mkdir()
    _run_env(d2, argv(2, "0"), **env)
    shutil.copy(d2 / "end", d2 / "start")
    shutil.copy(d2 / "end.json", d2 / "start.json")
    _run_env(d2, argv(2, "START"), **env)
    assert np.array_equal(np.load(d2 / "end"), full)
    with Phi4Lattice((64, 16, 32), dtau=0.01, m2=0.5, lam=1.5, seed=7, loops=10) as L:
        L.init_field(float(np.float32(np.sqrt(2 * 0.01))))
        for _ in range(4):
            assert L.run_frame()
        assert np.array_equal(L.download(), full)


def test_taumain_driver_double_well(gpu, tmp_path):
    """The taumain.py flow headless (stochquant_amd.driver): spawn, stream,
    parse; 199 values per frame, percent ends at 100, end file written."""
    from stochquant_amd.driver import TauhostRun
    frames = []
    with TauhostRun("double_well", frames=6, loops=200, cwd=str(tmp_path)) as run:
        for fr in run:
            frames.append(fr)
    assert run.returncode == 0, run.stderr
    assert len(frames) == 6 and frames[-1]["percent"] == pytest.approx(100.0)
    y = frames[-1]["y"]
    assert np.all(np.isfinite(y) | np.isneginf(y))   # -inf while no frame was stable yet (Δτ/Δt² = 5)
    assert frames[-1]["dtau"] <= 0.002
    assert (tmp_path / "V0_2e_0-8.txt").exists()


@pytest.mark.parametrize("C", ["1", "0"])
def test_configs0_phi4_32_through_tauhost(gpu, oracle_mod, tmp_path, C):
    """BASELINE configs[0] read literally: a 32^3 scalar
    φ⁴ lattice, Δτ = 0.01, 1000 Langevin steps through tauhost.o driven by
    taumain.py's 13-argument argv (one frame of loops = 1000; SQ_MODEL=phi4,
    SQ_SHAPE=32x32x32).  The end-file field equals the library run of the same
    frame bit for bit; with the noise off (C = 0) it equals the CPU oracle's
    1000 steps from the same start field bit for bit."""
    from stochquant_amd import Phi4Lattice, tauhost_argv
    env = dict(SQ_MODEL="phi4", SQ_SHAPE="32x32x32", SQ_SEED="24301")
    argv = tauhost_argv(32, 1.0, 0.01, 1, 0, C, 0, 1, 0, 1000, "0", "END", 16)[1:]
    out, _ = _run_env(tmp_path, argv, **env)
    assert len(out.strip().split("\n")) == 1
    cli = np.load(tmp_path / "end")
    assert cli.shape == (32, 32, 32)
    with Phi4Lattice((32, 32, 32), dtau=0.01, m2=1.0, lam=1.0, seed=24301, loops=1000, C=float(C)) as L:
        L.init_field(float(np.float32(np.sqrt(2 * 0.01))))
        phi0 = L.download()
        assert L.run_frame()
        lib = L.download()
    assert np.array_equal(cli, lib)
    if C == "0":
        p = oracle_mod.phi4_params((32, 32, 32), 0.01, 1.0, 1.0, 24301, C=0.0)
        ref = phi0
        for s in range(1000):
            ref = oracle_mod.phi4_step(p, ref, s)
        assert np.array_equal(cli, ref), f"max diff {np.max(np.abs(cli - ref))}"
