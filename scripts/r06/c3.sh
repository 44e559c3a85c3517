#!/bin/bash
# Round 6 call 3: the tolerance tests under the tightened bounds (TOL lines),
# then kernel traces of the slab path on one GPU (single / RCCL / P2P
# self-exchange, 320 steps after 400 warm-up) for the per-block budget.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c3}
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T "tests/test_gpu_phi4.py::test_noisy_step_within_tolerance" \
  "tests/test_gpu_phi4.py::test_full_size_256_one_step" "tests/test_gpu_phi4.py::test_stability_rule_quiet_on_stable_frames" \
  "tests/test_gpu_phi4.py::test_c2_hot_instance_vs_oracle" "tests/test_gpu_qm1d.py::test_frame_within_tolerance" \
  tests/test_gpu_fuzz.py > $O/t_tol.log 2>&1 || { tail -30 $O/t_tol.log; exit 3; }
tail -1 $O/t_tol.log
grep -o "TOL .*" $O/t_tol.log > $O/tol.txt || true
for c in single rccl p2p; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$c -o run -- python3 scripts/r06/slab_trace.py $c 320 \
    > $O/trace_$c.log 2>&1 || { tail -20 $O/trace_$c.log; exit 4; }
  cat $O/trace_$c.log | grep us/step
done
python3 scripts/r06/slab_budget.py $(find $O/tr_single -name "*kernel_trace.csv") $(find $O/tr_rccl -name "*kernel_trace.csv") \
  $(find $O/tr_p2p -name "*kernel_trace.csv") > $O/budget.txt 2>&1; tail -40 $O/budget.txt
timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_diag.log 2>&1 || { tail -20 $O/frames_diag.log; exit 5; }
cat $O/frames_diag.log
