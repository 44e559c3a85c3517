#!/bin/bash
# Slab-path schedules on one GPU (256^3, G = 16, RCCL / P2P self-exchange):
# core pairs K = 0, 1, 2, 4 with the rims on stream A or on the exchange stream.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/sched_ab
mkdir -p $O
for comm in ${COMMS:-rccl p2p}; do
  for cfg in "0 0" "1 0" "1 1" "2 0" "2 1" "4 0" "4 1"; do
    set -- $cfg
    SQ_GHOST=16 SQ_CORE_PAIRS=$1 SQ_RIMS_B=$2 timeout -k 10 100 python3 bench.py --comm $comm --steps 1600 --settle-ms 500 --no-cpu-baseline > $O/${comm}_k$1_b$2.log 2>&1 || exit 3
    python3 -c "
import json,sys
d=json.loads(open('$O/${comm}_k$1_b$2.log').read().strip().splitlines()[-1])
print('$comm K=$1 rimsB=$2', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
