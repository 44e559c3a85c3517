#!/bin/bash
# Round-4 call 19: the full GPU suite + smoke of the closing tree, then the
# driver's N = 1 invocation once.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c19}
mkdir -p $O
bash scripts/r04_suite.sh ${1:-r04_c19}/suite || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail $O/bench_driver.log; exit 4; }
grep -o '"value": [0-9.e+]*' $O/bench_driver.log | head -1
