#!/bin/bash
# Slab path on one GPU (RCCL self-exchange, 256^3): edges-first split on vs off, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_slab_ef}
mkdir -p $O
for r in 1 2; do
  for ef in 1 0; do
    SQ_EDGE_FIRST=$ef timeout -k 10 180 python bench.py --comm rccl --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check > $O/ef${ef}_$r.log 2>&1 || exit 2
    python3 -c "
import json
for l in open('$O/ef${ef}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); c=d['config']; print('edge_first=$ef round $r', round(d['ms_per_step']*1e3,3),'us/step', c.get('ghost_depth'), c.get('block_schedule'))
"
  done
done
