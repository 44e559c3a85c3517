#!/bin/bash
# Round-2 profile of the default bench command (256^3, fused two-step kernel):
# one rocprofv3 kernel-trace/stats run, then separate --pmc passes (FETCH_SIZE,
# WRITE_SIZE, SQ issue counters), each under its own hard time limit
# (MI355X_MICROARCH.md §rocprofv3 PMC slots).  Outputs under gpurun_out/prof_r02/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_r02
mkdir -p $O
B="bench.py --steps 400 --warmup 100 --settle-ms 300 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 2000 --no-cpu-baseline > $O/trace.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq -o run --output-format csv -- python3 $B > $O/sq.log 2>&1 || exit 5
echo done
