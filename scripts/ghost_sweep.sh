#!/bin/bash
# Ghost-zone depth sweep of the slab path on one GPU: prints "comm G ms_per_step value".
#   scripts/ghost_sweep.sh rccl "1 2 4 8 16"   |   scripts/ghost_sweep.sh loopback "1 4 8"
comm=$1; shift
for g in $1; do
  out=$(SQ_GHOST=$g timeout -k 10 120 python bench.py --comm "$comm" --slabs 2 --no-cpu-baseline --steps 2000) || exit 3
  echo "$out" | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$comm', $g, round(d['ms_per_step']*1e3, 3), '%.4g' % d['value'])"
done
