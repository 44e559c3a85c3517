#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_frdiag
mkdir -p $O
for p in 1 0; do
  for args in "2 1.0 0 4" "2 0.0 0 4" "2 1.0 1 4" "4 1.0 1 3"; do
    SQ_TB2_PIPE=$p timeout -k 10 120 python -u scripts/diag_fr_sites.py $args >> $O/p$p.log 2>&1 || exit 1
  done
done
tail -200 $O/p1.log $O/p0.log | cut -c1-400
