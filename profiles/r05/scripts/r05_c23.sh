#!/bin/bash
# Round 5, call 23: the split-barrier C1 kernel with the polling wave at priority
# 3, sleeping between polls (SQ_QM1D_PSLEEP=1) or not (0), against the plain
# kernel (SQ_QM1D_PIPE=0), interleaved twice; stamps of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c23}
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_qm1d.py -k "grid" > $O/qm1d.log 2>&1 || { tail -30 $O/qm1d.log; exit 3; }
tail -1 $O/qm1d.log
for r in 1 2; do
  for cfg in "1 1" "1 0" "0 1"; do
    set -- $cfg
    SQ_QM1D_PIPE=$1 SQ_QM1D_PSLEEP=$2 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_p$1_s$2_$r.log 2>&1 || { tail -5 $O/c1_p$1_s$2_$r.log; exit 4; }
    echo "pipe=$1 psleep=$2 run=$r $(grep '^{' $O/c1_p$1_s$2_$r.log)"
  done
done
for cfg in "1 1" "1 0"; do
  set -- $cfg
  rm -f $O/stamps_s$2.txt
  SQ_QM1D_PIPE=$1 SQ_QM1D_PSLEEP=$2 SQ_QM1D_STAMPS=$O/stamps_s$2.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st_s$2.log 2>&1 || exit 5
  echo "stamps psleep=$2"; python3 scripts/c1_stamps.py $O/stamps_s$2.txt
done
