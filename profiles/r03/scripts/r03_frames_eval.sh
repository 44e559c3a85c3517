#!/bin/bash
# Frame kernel change: GPU phi4 tests (all), frame rows, kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_feval}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f.log 2>&1 || { cat $O/rows_f.log; exit 3; }
grep f1 $O/rows_f.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/frames_only.py > $O/prof.log 2>&1 || { tail $O/prof.log; exit 4; }
head -4 $O/prof/run_kernel_stats.csv
