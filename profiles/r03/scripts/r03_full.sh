#!/bin/bash
# Full GPU suite + frame rows + default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f.log 2>&1 || { cat $O/rows_f.log; exit 3; }
grep f1 $O/rows_f.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 4; }
tail -1 $O/bench.log
