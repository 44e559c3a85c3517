#!/bin/bash
# Snake block order x store policy at 512^3 / 1024^3 / 256^3, interleaved.  Prints "size snake pf us_per_step".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for round in 1 2; do
  for size in 512 1024 256; do
    steps=400; [ $size = 1024 ] && steps=60; [ $size = 256 ] && steps=2000
    for sn in 0 1; do
      for pf in 3 4; do
        out=$(SQ_SNAKE=$sn SQ_PREFETCH=$pf timeout -k 10 120 python bench.py --size $size --steps $steps --warmup 100 --no-cpu-baseline) || exit 3
        echo "$out" | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($size, $sn, $pf, round(d['ms_per_step']*1e3, 2))"
      done
    done
  done
done
