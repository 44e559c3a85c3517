#!/bin/bash
# Step s+1 two planes behind (SQ_TB2_LAG=1): bitwise phi4 tests with it forced,
# then an interleaved A/B of the 256^3 bench line against the round-2 kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_lag}
mkdir -p $O
SQ_TB2_LAG=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py > $O/tests_lag.log 2>&1 || { tail -30 $O/tests_lag.log; exit 2; }
tail -1 $O/tests_lag.log
for r in 1 2 3; do
  for q in 0 1; do
    SQ_TB2_LAG=$q timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-c3 --no-check > $O/b_lag${q}_$r.log 2>&1 || { tail $O/b_lag${q}_$r.log; exit 3; }
    python3 -c "
import json
for l in open('$O/b_lag${q}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('lag=$q round $r', round(d['ms_per_step']*1e3,3),'us/step wall', r['avg_step_us'], 'kernel busy', r.get('busy_fraction'))
"
  done
done
