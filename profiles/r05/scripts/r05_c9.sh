#!/bin/bash
# Round 5, call 9: C1 sweep of barrier form x sites per thread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c9}
mkdir -p $O
for r in 1 2; do for cfg in "1 4" "3 4" "3 2" "1 2" "3 8"; do
  set -- $cfg
  SQ_QM1D_BAR=$1 SQ_QM1D_GK=$2 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_bar$1_k$2_$r.log 2>&1 || { tail -5 $O/c1_bar$1_k$2_$r.log; exit 4; }
  echo "bar=$1 K=$2 run=$r $(grep '^{' $O/c1_bar$1_k$2_$r.log)"
done; done
for cfg in "3 4" "3 2"; do
  set -- $cfg
  rm -f $O/stamps_bar$1_k$2.txt
  SQ_QM1D_BAR=$1 SQ_QM1D_GK=$2 SQ_QM1D_STAMPS=$O/stamps_bar$1_k$2.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st.log 2>&1 || exit 5
  echo "bar=$1 K=$2"; python3 scripts/c1_stamps.py $O/stamps_bar$1_k$2.txt
done
