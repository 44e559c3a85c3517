#!/bin/bash
# Slab path on one GPU (self-exchange, 256^3, measured ghost depth): RCCL and
# P2P transports, two rounds, then a kernel trace of the RCCL run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_slab}
mkdir -p $O
for r in 1 2; do
  for c in rccl p2p; do
    timeout -k 10 180 python bench.py --comm $c --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check > $O/b_${c}_$r.log 2>&1 || exit 2
  done
done
for f in $O/b_*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; c=d['config']; print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step', c.get('ghost_depth'), c.get('block_schedule'))
"; done
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --comm rccl --steps 320 --warmup 50 --settle-ms 300 --no-cpu-baseline --no-c3 --no-check > $O/trace.log 2>&1 || exit 3
python3 scripts/slab_timeline.py $O/trace/run_kernel_trace.csv 60 > $O/timeline.txt || exit 4
tail -25 $O/timeline.txt
