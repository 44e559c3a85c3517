#!/bin/bash
# Round-3 start: GPU tests, the driver's bench invocation, 2000 steps, 512^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_base
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_2000.log 2>&1 || exit 3
timeout -k 10 150 python3 bench.py --size 512 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_512.log 2>&1 || exit 4
grep -h '^{' $O/bench_driver.log $O/bench_2000.log $O/bench_512.log | cut -c1-600
echo done
