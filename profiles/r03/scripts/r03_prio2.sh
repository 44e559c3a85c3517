#!/bin/bash
# Wave priority by march progress (SQ_TB2_PRIO=1) vs off, 256^3 and 512^3, two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_prio2}
mkdir -p $O
B="bench.py --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check"
for r in 1 2; do
  for p in 1 2; do
    SQ_TB2_PRIO=$p timeout -k 10 120 python $B > $O/b256_p${p}_$r.log 2>&1 || exit 2
    SQ_TB2_PRIO=$p timeout -k 10 120 python bench.py --size 512 --steps 200 --warmup 20 --settle-ms 800 --no-cpu-baseline --no-check > $O/b512_p${p}_$r.log 2>&1 || exit 3
  done
done
for f in $O/b*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step', '%.3e'%d['value'], r['avg_launch_us'])
"; done
