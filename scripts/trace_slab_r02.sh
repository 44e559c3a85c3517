#!/bin/bash
# Kernel timeline of the slab path (RCCL self-exchange, 256^3, G = 16): one
# rocprofv3 kernel trace of a short bench, for the per-launch breakdown
# (scripts/slab_timeline.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/trace_slab
mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --comm ${1:-rccl} --steps 320 --warmup 50 --settle-ms 300 --no-cpu-baseline > $O/bench.log 2>&1 || exit 2
find $O -name "*kernel_trace.csv" | head -3
