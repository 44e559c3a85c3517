#!/bin/bash
# Where the slab path's time goes: rocprofv3 kernel trace of the RCCL
# self-exchange bench (256^3, deep halo), then the bench at pinned ghost depths.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_slab_r02
mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --comm rccl --steps 800 --warmup 100 --settle-ms 500 --no-cpu-baseline > $O/trace.log 2>&1 || exit 2
for g in 16 32 64; do
  SQ_GHOST=$g timeout -k 10 120 python3 bench.py --comm rccl --steps 1600 --warmup 200 --no-cpu-baseline > $O/ghost_$g.log 2>&1 || exit 3
done
timeout -k 10 120 python3 bench.py --steps 1600 --warmup 200 --no-cpu-baseline > $O/single.log 2>&1 || exit 4
echo done
