#!/bin/bash
# Round 5, call 20: balancing the two blocks of a CU -- the second-dispatched
# block takes its priority quarters SQ_TB2_PSHIFT planes later, or
# SQ_TB2_PRIO=3 (priority by the other block's progress, per-CU words),
# interleaved twice against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c20}
mkdir -p $O
for r in 1 2; do
  for cfg in "1 0" "1 2" "1 4" "3 0"; do
    set -- $cfg
    SQ_TB2_PRIO=$1 SQ_TB2_PSHIFT=$2 timeout -k 10 120 python3 scripts/ab_tb2_balance.py > $O/p$1_s$2_$r.log 2>&1 || { tail -5 $O/p$1_s$2_$r.log; exit 3; }
    grep '^{' $O/p$1_s$2_$r.log
  done
done
