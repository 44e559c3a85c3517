#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_qgk; mkdir -p $O
for k in 8 16 32; do
  SQ_QM1D_GK=$k timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py -k "grid_frame or large_chain" > $O/tests_$k.log 2>&1 || { tail -20 $O/tests_$k.log; exit 2; }
  SQ_QM1D_GK=$k timeout -k 10 200 python -u scripts/bench_qm1d.py --ordering jacobi --no-cpu > $O/bench_$k.log 2>&1 || exit 3
  echo "K=$k $(tail -1 $O/tests_$k.log) $(tail -1 $O/bench_$k.log)"
done
