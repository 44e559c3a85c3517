#!/bin/bash
# Round 5, call 3: does hipExtAnyOrderLaunch overlap consecutive kernels on
# gfx950 (scripts/anyorder_probe.hip)?  Then the default bench (2000 steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c3}
mkdir -p $O
timeout -k 10 60 ./scripts/bin/anyorder_probe 512 2000 > $O/anyorder.log 2>&1 || { cat $O/anyorder.log; exit 2; }
timeout -k 10 60 ./scripts/bin/anyorder_probe 1024 2000 >> $O/anyorder.log 2>&1 || { cat $O/anyorder.log; exit 3; }
cat $O/anyorder.log
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 4; }
