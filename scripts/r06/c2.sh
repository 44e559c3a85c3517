#!/bin/bash
# Round 6 call 2: sticky gate + noise-protocol tests, the tolerance tests with
# their measured maxima printed (TOL lines), the C = 1 oracle digests made on
# the box (device Box-Muller tables), the full-size noise check against them,
# then the driver's bench at N = 1 and the N = 8 shape on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/${1:-r06_c2}
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $T "tests/test_gpu_phi4.py::test_gate_timeout_is_sticky" \
  "tests/test_gpu_phi4.py::test_oracle_protocol_noise_matches_device_oracle" > $O/t_new.log 2>&1 \
  || { tail -30 $O/t_new.log; exit 2; }
tail -1 $O/t_new.log
timeout -k 10 600 $T "tests/test_gpu_phi4.py::test_noisy_step_within_tolerance" \
  "tests/test_gpu_phi4.py::test_full_size_256_one_step" "tests/test_gpu_phi4.py::test_full_size_512" \
  "tests/test_gpu_phi4.py::test_c5_slab_1024x1024x128_rccl" "tests/test_gpu_phi4.py::test_full_size_256_rccl_slab_fused_vs_oracle" \
  "tests/test_gpu_phi4.py::test_stability_rule_quiet_on_stable_frames" "tests/test_gpu_phi4.py::test_c2_hot_instance_vs_oracle" \
  "tests/test_gpu_qm1d.py::test_frame_within_tolerance" tests/test_gpu_fuzz.py > $O/t_tol.log 2>&1 \
  || { tail -30 $O/t_tol.log; exit 3; }
tail -1 $O/t_tol.log
grep "^TOL" $O/t_tol.log > $O/tol.txt || true
timeout -k 10 300 python -u tests/golden/make_oracle_slabs.py --noise --threads 16 --out $O/oracle_slabs.json \
  > $O/make_noise.log 2>&1 || { tail -20 $O/make_noise.log; exit 4; }
cp $O/oracle_slabs.json tests/golden/oracle_slabs.json
timeout -k 10 200 $T "tests/test_gpu_phi4.py::test_oracle_check_noise_full_size_256" > $O/t_full.log 2>&1 \
  || { tail -30 $O/t_full.log; exit 5; }
tail -1 $O/t_full.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.log 2>&1 || { tail -20 $O/bench_n1.log; exit 6; }
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 > $O/bench_n8.log 2>&1 \
  || { tail -20 $O/bench_n8.log; exit 7; }
python3 - <<PY
import json
for n in ("n1", "n8"):
    d = json.loads([l for l in open("$O/bench_%s.log" % n) if l.startswith("{")][-1])
    print(n, {k: d.get(k) for k in ("value", "n_gpus", "ms_per_step", "multi_rank_check", "oracle_check", "oracle_check_noise", "transport_fallback", "error")})
    c5 = d.get("c5_1024", {})
    print(n, "c5", {k: c5.get(k) for k in ("value", "multi_rank_check", "oracle_check", "oracle_check_noise", "error")})
    if n == "n1":
        print("frames", d["frames_256"].get("overhead"), "slab", d["slab_1gpu"]["rccl"].get("ratio_to_single"), d["slab_1gpu"]["p2p"].get("ratio_to_single"))
PY
