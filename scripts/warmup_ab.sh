#!/bin/bash
# bench value vs warm-up length on one box (clock ramp check).  Prints "warmup value ms_per_step".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for w in 200 2000 200 2000 10000 200; do
  out=$(timeout -k 10 120 python bench.py --no-cpu-baseline --warmup $w) || exit 3
  echo "$out" | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['warmup'], '%.4g' % d['value'], round(d['ms_per_step']*1e3, 3))"
done
