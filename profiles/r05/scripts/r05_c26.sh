#!/bin/bash
# Round 5, call 26: age-order arbitration only (SQ_TB2_PRIO=0) with the first-
# dispatched block of each CU given more planes (SQ_TB2_ZSPLIT=d: chunks 16+d /
# 16-d), against the default (progress priority, even chunks), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c26}
mkdir -p $O
for r in 1 2; do
  for cfg in "1 0" "0 0" "0 4" "0 6" "0 8" "0 10"; do
    set -- $cfg
    SQ_TB2_PRIO=$1 SQ_TB2_ZSPLIT=$2 timeout -k 10 120 python3 scripts/ab_tb2_balance.py > $O/p$1_z$2_$r.log 2>&1 || { tail -5 $O/p$1_z$2_$r.log; exit 3; }
    grep '^{' $O/p$1_z$2_$r.log
  done
done
