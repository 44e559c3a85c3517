#!/bin/bash
# Round 6 call 19: per-pair block stamps of the resident march (where its
# extra ~3 us per pair goes), prio by quarter and off; and one pair per
# resident launch (the hand-off forms' own cost without the dataflow).
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c19}
mkdir -p $O
timeout -k 10 200 python3 -u scripts/r06/run_stamps.py 8 1 > $O/stamps_prio1.log 2>&1 || { tail -30 $O/stamps_prio1.log; exit 3; }
grep -v "amdgpu.ids" $O/stamps_prio1.log
timeout -k 10 200 python3 -u scripts/r06/run_stamps.py 8 0 > $O/stamps_prio0.log 2>&1 || { tail -30 $O/stamps_prio0.log; exit 4; }
grep -v "amdgpu.ids" $O/stamps_prio0.log
timeout -k 10 300 python3 -u scripts/r06/run_ab.py 4 maxp > $O/run_ab_maxp.log 2>&1 || { tail -30 $O/run_ab_maxp.log; exit 5; }
grep -v "^round\|amdgpu.ids" $O/run_ab_maxp.log
timeout -k 10 300 python3 -u scripts/r06/run_ab.py 4 maxp_acq > $O/run_ab_maxp_acq.log 2>&1 || { tail -30 $O/run_ab_maxp_acq.log; exit 6; }
grep -v "^round\|amdgpu.ids" $O/run_ab_maxp_acq.log
