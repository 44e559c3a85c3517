#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_qbar; mkdir -p $O
for b in 1 0; do
  SQ_QM1D_BAR=$b timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gpu_qm1d.py -k "grid_frame or large_chain or ho_noiseless" > $O/tests_$b.log 2>&1 || { tail -20 $O/tests_$b.log; exit 2; }
  SQ_QM1D_BAR=$b timeout -k 10 120 python -u scripts/bench_qm1d.py --ordering jacobi --no-cpu > $O/bench_$b.log 2>&1 || exit 3
  echo "BAR=$b $(tail -1 $O/tests_$b.log) $(tail -1 $O/bench_$b.log)"
done
