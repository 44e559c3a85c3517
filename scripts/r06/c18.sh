#!/bin/bash
# Round 6 call 18: the resident march's wave priority (by quarter of the pair,
# as the per-pair kernel, or off) for both load forms, against pair launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c18}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/r06/run_ab.py 6 > $O/run_ab_sc1.log 2>&1 || { tail -30 $O/run_ab_sc1.log; exit 3; }
grep -v "^round\|amdgpu.ids" $O/run_ab_sc1.log
timeout -k 10 300 python3 -u scripts/r06/run_ab.py 6 acq > $O/run_ab_acq.log 2>&1 || { tail -30 $O/run_ab_acq.log; exit 4; }
grep -v "^round\|amdgpu.ids" $O/run_ab_acq.log
