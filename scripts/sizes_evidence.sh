#!/bin/bash
# rocprofv3 kernel stats and PMC traffic (FETCH_SIZE / WRITE_SIZE, one counter
# per pass) of the 512^3 (C3) bench command, and kernel stats of the RCCL
# self-exchange slab path at 256^3; outputs under gpurun_out/sizes_ev/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/sizes_ev
mkdir -p $O
B="bench.py --size 512 --steps 100 --warmup 20 --settle-ms 300 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/trace512 -o run --output-format csv -- python3 $B > $O/trace512.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch512 -o run --output-format csv -- python3 $B > $O/fetch512.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write512 -o run --output-format csv -- python3 $B > $O/write512.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/trace_rccl -o run --output-format csv -- python3 bench.py --comm rccl --steps 800 --warmup 100 --settle-ms 300 --no-cpu-baseline > $O/trace_rccl.log 2>&1 || exit 5
echo done
