#!/bin/bash
# Device-controlled frames: the GPU frame tests, then the frame-overhead rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_fdev}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "run_frames or stability or snapshot or frame or rollback or checkpoint" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -3 $O/tests.log
timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f.log 2>&1 || { cat $O/rows_f.log; exit 3; }
cat $O/rows_f.log
