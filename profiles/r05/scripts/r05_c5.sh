#!/bin/bash
# Round 5, call 5: the QM1D grid kernel's sc1 hand-off barrier -- bitwise
# tests first (grid vs one-CU for every barrier form, C1 frames, the oracle,
# the timeout), then C1 timing A/B against the fenced barrier.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c5}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 120 $T tests/test_gpu_qm1d.py::test_grid_barrier_timeout_returns_error > $O/barrier.log 2>&1 || { tail -30 $O/barrier.log; exit 2; }
timeout -k 10 400 $T tests/test_gpu_qm1d.py -k "grid or large_chain" > $O/qm1d_grid.log 2>&1 || { tail -30 $O/qm1d_grid.log; exit 3; }
tail -2 $O/qm1d_grid.log
for r in 1 2; do for b in 2 1; do
  SQ_QM1D_BAR=$b timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_bar${b}_$r.log 2>&1 || { tail -5 $O/c1_bar${b}_$r.log; exit 4; }
  echo "bar=$b run=$r $(cat $O/c1_bar${b}_$r.log)"
done; done
