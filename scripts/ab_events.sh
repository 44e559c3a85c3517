#!/bin/bash
# Wall time of the driver's short invocation with and without the hipEvent
# pair that times the kernel region (what the two markers cost in `value`).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab_events
mkdir -p $O
for i in 1 2 3; do
  for mode in ev noev; do
    extra=""; [ $mode = noev ] && extra="--no-profile-events"
    timeout -k 10 100 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $extra > $O/${mode}_$i.log 2>&1 || exit 3
    python3 -c "
import json
d=json.loads(open('$O/${mode}_$i.log').read().strip().splitlines()[-1])
print('$mode $i', round(d['ms_per_step']*1e3,2), 'us/step wall', d['roofline']['avg_step_us'])"
  done
done
