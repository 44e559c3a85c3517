#!/bin/bash
# Round 5, call 8: QM1D grid kernel with the field in registers and the
# post-barrier loads batched -- bitwise tests, then C1 timing and stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c8}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 120 $T tests/test_gpu_qm1d.py -k barrier_timeout > $O/barrier.log 2>&1 || { tail -30 $O/barrier.log; exit 2; }
timeout -k 10 400 $T tests/test_gpu_qm1d.py tests/test_gpu_tauhost.py::test_config_c1_chain_through_tauhost > $O/qm1d.log 2>&1 || { tail -30 $O/qm1d.log; exit 3; }
tail -2 $O/qm1d.log
for r in 1 2; do for cfg in "1 8" "3 8" "3 4"; do
  set -- $cfg
  SQ_QM1D_BAR=$1 SQ_QM1D_GK=$2 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_bar$1_k$2_$r.log 2>&1 || { tail -5 $O/c1_bar$1_k$2_$r.log; exit 4; }
  echo "bar=$1 K=$2 run=$r $(grep '^{' $O/c1_bar$1_k$2_$r.log)"
done; done
for b in 1 3; do
  rm -f $O/stamps_bar$b.txt
  SQ_QM1D_BAR=$b SQ_QM1D_STAMPS=$O/stamps_bar$b.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st_bar$b.log 2>&1 || { tail -5 $O/st_bar$b.log; exit 5; }
  echo "bar=$b"; python3 scripts/c1_stamps.py $O/stamps_bar$b.txt
done
