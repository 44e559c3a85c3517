#!/bin/bash
# Round 6 call 10: do back-to-back launches on one stream overlap?
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c10}
mkdir -p $O
timeout -k 10 60 ./scripts/r06/overlap_probe > $O/overlap_probe.log 2>&1 || { tail -20 $O/overlap_probe.log; exit 2; }
cat $O/overlap_probe.log
