"""bench.py's roofline object on CPU: the committed PMC
record is used only when its build id, kernel instance and grid are the ones
this run launched; a mismatched record gives `frac: null` and
`stale_profile: true`, and runs without a record (slab paths, N > 1, other
lattices) are labelled `hbm_algorithmic` in GB/s -- never "valu" beside a
byte ratio.  The lattice is a stand-in; no GPU call is made."""
import argparse
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HOT = "phi4_tb2_kernel<true, false, 1, false, true, false>"


class _Lat:
    kernel_name = "phi4_tb2_kernel<true> (2 steps per launch) one round of 512 blocks"

    def __init__(self, kernel=HOT, grid=327680):
        self._info = {"kernel": kernel, "grid": grid, "launches": 10}

    def launch_info(self):
        return dict(self._info)

    def step(self, n):
        pass

    def block_stamps(self):
        st = np.arange(512, dtype=np.int64)
        return st, st + 3000

    def block_clocks(self):
        st = np.arange(512, dtype=np.int64)
        return st, st + 3000 * 21


PERF = {"steps": 20, "kernel_launches": 10, "fused_steps": 20, "step_kernel_launches": 20, "step_kernel_ms": 0.33}


def _profile(tmp_path, build, kernel=HOT, grid=327680, rocprof_us=32.2):
    rec = {"kernel": f"void sq::(anonymous namespace)::{kernel}(sq::Phi4StepArgs)", "grid": grid,
           "build_id_phi4": build, "valu_busy_cycles_per_launch": 59187200.0, "hbm_bytes_per_launch": 151132160.0,
           "rocprof_avg_us": rocprof_us, "rocprof_median_us": rocprof_us}
    p = tmp_path / "driver_profile.json"
    p.write_text(json.dumps({"command": "python3 bench.py --steps 20 --warmup 5", "configs": {"256": rec}}))
    return str(p)


def _roofline(monkeypatch, tmp_path, lat, profile, world=1, slab=False):
    import bench
    monkeypatch.setattr(bench, "PROFILE", profile)
    a = argparse.Namespace(steps=20, strong=False)
    rl, _, fused = bench.roofline(a, lat, 256, world, slab, 0.00033, dict(PERF), 1, 256 ** 3)
    return rl


@pytest.fixture
def build(sqlib):
    from stochquant_amd import _lib
    return _lib.build_id()


def test_matching_record_gives_the_valu_fraction(monkeypatch, tmp_path, build):
    rl = _roofline(monkeypatch, tmp_path, _Lat(), _profile(tmp_path, build["phi4"]))
    assert rl["bound"] == "valu" and rl["unit"].startswith("G VALU")
    assert 0 < rl["frac"] <= 1 and rl["traffic"] == 151132160.0
    assert rl["kernel"] == HOT and rl["grid_threads"] == 327680 and rl["build_id"] == build
    assert "stale_profile" not in rl


@pytest.mark.parametrize("what", ["build", "kernel", "grid"])
def test_mismatched_record_is_refused(monkeypatch, tmp_path, build, what):
    kw = {"build": dict(build="0123456789abcdef"), "kernel": dict(kernel="phi4_tb2_kernel<true, false, 6, true, true, false>"),
          "grid": dict(grid=163840)}[what]
    prof = _profile(tmp_path, kw.get("build", build["phi4"]), kernel=kw.get("kernel", HOT), grid=kw.get("grid", 327680))
    rl = _roofline(monkeypatch, tmp_path, _Lat(), prof)
    assert rl["frac"] is None and rl["stale_profile"] is True and rl["achieved"] is None
    assert what in rl["stale_reason"]
    assert rl["traffic"] is None
    assert rl["frac_algorithmic"] > 0          # the contract's byte ratio still reported beside it
    assert "frac_at_measured_clock" not in rl


def test_no_record_is_labelled_algorithmic(monkeypatch, tmp_path, build):
    """N > 1 / slab paths: no PMC record -> bound 'hbm_algorithmic', GB/s."""
    prof = _profile(tmp_path, build["phi4"])
    for world, slab in ((2, True), (1, True)):
        rl = _roofline(monkeypatch, tmp_path, _Lat(), prof, world=world, slab=slab)
        assert rl["bound"] == "hbm_algorithmic" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
        assert rl["frac"] == rl["frac_algorithmic"]
    missing = str(tmp_path / "none.json")
    rl = _roofline(monkeypatch, tmp_path, _Lat(), missing)
    assert rl["bound"] == "hbm_algorithmic" and "stale_profile" not in rl


def test_committed_profile_describes_this_build(build):
    """The committed record bench.py reads carries the build id and kernel it
    was taken from (a record without them can never be used)."""
    import bench
    path = os.path.join(ROOT, bench.PROFILE)
    if not os.path.exists(path):
        pytest.skip("no profile committed for this round yet")
    rec = json.load(open(path))["configs"]["256"]
    assert rec.get("build_id_phi4") and bench.short_kernel(rec["kernel"]) == HOT


@pytest.mark.parametrize("rocprof_us,mismatch", [(32.2, False), (33.9, False), (35.0, True), (30.0, True)])
def test_profile_timing_mismatch_is_flagged(monkeypatch, tmp_path, build, rocprof_us, mismatch):
    """a record whose rocprof launch time is more than 3 %
    off this run's live launch (33.0 us here) is flagged and its durations are
    not quoted; the clock-independent counts still divide the live time."""
    rl = _roofline(monkeypatch, tmp_path, _Lat(), _profile(tmp_path, build["phi4"], rocprof_us=rocprof_us))
    assert rl["profile_timing_mismatch"] is mismatch
    assert rl["launch_us_vs_rocprof_avg"] == round(33.0 / rocprof_us, 4)
    assert ("profile_rocprof_avg_us" in rl) is (not mismatch)
    assert ("profile_rocprof_median_us" in rl) is (not mismatch)
    # frac_hbm_real and the VALU fraction come from the live launch time either way
    assert rl["frac_hbm_real"] == round(151132160.0 / 33e-6 / 1e9 / 8000.0, 4)
    assert rl["frac"] == round(59187200.0 / 33e-6 / 1e9 / (1024 * 2.4), 4)
