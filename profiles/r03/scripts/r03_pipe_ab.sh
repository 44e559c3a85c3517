#!/bin/bash
# A/B of the fused kernel: SQ_TB2_PIPE=0 (round-2 kernel) vs 1 (pipelined), after the GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_pipe}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="bench.py --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline"
for r in 1 2; do
  for p in 0 1; do
    SQ_TB2_PIPE=$p timeout -k 10 120 python $B > $O/b256_p${p}_$r.log 2>&1 || exit 2
    SQ_TB2_PIPE=$p timeout -k 10 120 python bench.py --size 512 --steps 200 --warmup 20 --settle-ms 800 --no-cpu-baseline > $O/b512_p${p}_$r.log 2>&1 || exit 3
  done
done
for f in $O/b*.log; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step', '%.3e'%d['value'], r['avg_launch_us'], r['kernel'][:40])
"; done
