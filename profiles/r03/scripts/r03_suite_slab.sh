#!/bin/bash
# Full GPU suite, then the slab path with the in-kernel edges-done signal vs the event (SQ_EDGE_FLAG=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_ss}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 2; }
tail -1 $O/suite.log
for r in 1 2; do
  for f in 1 0; do
    SQ_EDGE_FLAG=$f timeout -k 10 180 python bench.py --comm rccl --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check > $O/rccl_f${f}_$r.log 2>&1 || exit 3
    SQ_EDGE_FLAG=$f timeout -k 10 180 python bench.py --comm p2p --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check > $O/p2p_f${f}_$r.log 2>&1 || exit 4
  done
done
for f in $O/rccl_*.log $O/p2p_*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step')
"; done
