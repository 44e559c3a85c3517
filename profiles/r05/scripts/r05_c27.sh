#!/bin/bash
# Round 5, call 27 (diagnostic build): is the frame instances' VGPR cap
# (waves_per_eu 6) part of their cost?  Raw 256^3 steps with the raw instance
# as built (waves_per_eu 1) and under the cap (SQ_TB2_RAW6=1), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c27}
mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    if [ $v = 1 ]; then export SQ_TB2_RAW6=1; else unset SQ_TB2_RAW6; fi
    timeout -k 10 120 python3 scripts/ab_tb2_balance.py > $O/raw6_${v}_$r.log 2>&1 || { tail -5 $O/raw6_${v}_$r.log; exit 3; }
    echo "raw6=$v $(grep '^{' $O/raw6_${v}_$r.log)"
  done
done
