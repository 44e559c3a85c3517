#!/bin/bash
# A/B of the deep-halo last-step edge split on one GPU (RCCL self-exchange and
# 2 loopback slabs), interleaved rounds.  Prints "comm edge_first G us_per_step".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for round in 1 2 3; do
  for comm in rccl loopback; do
    for ef in 0 1; do
      for g in 4 16; do
        out=$(SQ_EDGE_FIRST=$ef SQ_GHOST=$g timeout -k 10 120 python bench.py --comm $comm --slabs 2 --no-cpu-baseline --steps 1600) || exit 3
        echo "$out" | tail -n 1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$comm', $ef, $g, round(d['ms_per_step']*1e3, 3))"
      done
    done
  done
done
