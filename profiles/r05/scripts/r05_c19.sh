#!/bin/bash
# Round 5, call 19: balancing the two fused-kernel blocks on a CU (the second
# dispatched runs 8 % longer): round-biased wave priority (SQ_TB2_PRIO=2) and
# uneven chunk pairs (SQ_TB2_ZSPLIT=d), interleaved twice against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c19}
mkdir -p $O
for r in 1 2; do
  for cfg in "1 0" "2 0" "1 1" "1 2" "2 1"; do
    set -- $cfg
    SQ_TB2_PRIO=$1 SQ_TB2_ZSPLIT=$2 timeout -k 10 120 python3 scripts/ab_tb2_balance.py > $O/p$1_z$2_$r.log 2>&1 || { tail -5 $O/p$1_z$2_$r.log; exit 3; }
    grep '^{' $O/p$1_z$2_$r.log
  done
done
