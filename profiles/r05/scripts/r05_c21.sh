#!/bin/bash
# Round 5, call 21: SQ_TB2_PRIO=3 -- wave priority by the other block's
# progress through two claimed words per CU -- against the default, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c21}
mkdir -p $O
for r in 1 2; do
  for p in 1 3; do
    SQ_TB2_PRIO=$p timeout -k 10 120 python3 scripts/ab_tb2_balance.py > $O/p${p}_$r.log 2>&1 || { tail -5 $O/p${p}_$r.log; exit 3; }
    grep '^{' $O/p${p}_$r.log
  done
done
