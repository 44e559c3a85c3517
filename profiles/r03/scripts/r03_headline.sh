#!/bin/bash
# Headline evidence: smoke(), the driver's own bench invocation twice, 1024^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_head}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || exit 3
done
timeout -k 10 300 python bench.py --size 1024 --steps 40 --warmup 10 --no-cpu-baseline --no-c3 --no-check > $O/bench_1024.log 2>&1 || exit 4
for f in $O/bench_*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], '%.3e'%d['value'], round(d['ms_per_step']*1e3,3), 'us/step frac', r['frac'], 'frac_wall', r.get('frac_wall'), 'busy', r.get('busy_fraction'), 'c3', '%.3e'%d['c3_512']['value'] if 'c3_512' in d else None, d.get('multi_rank_check'))
"; done
