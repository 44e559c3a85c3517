#!/bin/bash
# Round-4 call 18: under the power cap, does a tile with less first-step
# redundancy pay at one block per CU?  256^3, 2000 steps, interleaved:
# default (16-plane chunks, 512 blocks, 2 per CU, redundancy 1.203), 32-plane
# chunks (256 blocks, one per CU, 1.164) with the block barrier and with the
# neighbour sync (a lone block's barrier waits are not filled by another).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c18}
mkdir -p $O
B="--steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for r in 1 2; do for cfg in "def - barrier" "z32 32 barrier" "z32p 32 p2p" "z24 24 barrier"; do
  set -- $cfg
  if [ "$2" = "-" ]; then unset SQ_FUSE2_Z; else export SQ_FUSE2_Z=$2; fi
  SQ_TB2_SYNC=$3 timeout -k 10 180 python3 bench.py $B > $O/b_$1_$r.log 2>&1 || { tail $O/b_$1_$r.log; exit 2; }
  echo "$1 run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/b_$1_$r.log) $(grep -o '"clock_MHz_measured": [0-9.]*' $O/b_$1_$r.log) $(grep -o '"busy_fraction": [0-9.]*' $O/b_$1_$r.log)"
done; done
