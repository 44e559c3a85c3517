#!/bin/bash
# Round 5, call 6: the QM1D grid kernel's flag barrier (SQ_QM1D_BAR=3) --
# bitwise tests first, then C1 timing against the counter barrier at 8, 4, 2
# sites per thread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c6}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 120 $T tests/test_gpu_qm1d.py -k barrier_timeout > $O/barrier.log 2>&1 || { tail -30 $O/barrier.log; exit 2; }
timeout -k 10 400 $T tests/test_gpu_qm1d.py -k "grid or large_chain" > $O/qm1d_grid.log 2>&1 || { tail -30 $O/qm1d_grid.log; exit 3; }
tail -2 $O/qm1d_grid.log
for r in 1 2; do for cfg in "1 8" "3 8" "3 4" "3 2"; do
  set -- $cfg
  SQ_QM1D_BAR=$1 SQ_QM1D_GK=$2 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_bar$1_k$2_$r.log 2>&1 || { tail -5 $O/c1_bar$1_k$2_$r.log; exit 4; }
  echo "bar=$1 K=$2 run=$r $(grep '^{' $O/c1_bar$1_k$2_$r.log)"
done; done
