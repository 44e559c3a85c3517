#!/bin/bash
# Round 6 call 17: the resident two-step march (SQ_TB2_RUN=1,
# csrc/sq_phi4_run.hip) -- its bitwise GPU tests, one repeat of the hot-path
# parity tests, then an interleaved A/B against one launch per pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c17}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_run.py > $O/tests_run.log 2>&1 || { tail -40 $O/tests_run.log; exit 2; }
tail -1 $O/tests_run.log
timeout -k 10 300 python3 -u scripts/r06/run_ab.py 6 > $O/run_ab.log 2>&1 || { tail -30 $O/run_ab.log; exit 3; }
grep -v "^round" $O/run_ab.log
