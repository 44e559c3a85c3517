#!/bin/bash
# Round 5, call 2: the driver-command profile of the current build (the record
# bench.py's roofline reads, stamped with the build id), a two-rank P2P bench
# line on one GPU (N > 1 labels, oracle_check at N = 2), and a kernel trace of
# the batched frames with the per-launch-index breakdown.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c2}
mkdir -p $O
bash scripts/r05_driver_prof.sh r05_c2/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 2; }
tail -4 $O/prof.log
timeout -k 10 300 python3 bench.py --gpus 2 --same-device --comm p2p --steps 20 --warmup 5 > $O/p2p_2ranks.log 2>&1 || { tail -20 $O/p2p_2ranks.log; exit 3; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/ftrace -o run --output-format csv -- python3 scripts/bench_rows_f.py > $O/rows_f.log 2>&1 || { tail -20 $O/rows_f.log; exit 4; }
python3 scripts/frame_timeline.py $(find $O/ftrace -name '*kernel_trace.csv' | head -1) > $O/frame_timeline.txt 2>&1 || exit 5
find $O/ftrace -name '*kernel_trace.csv' -delete
cat $O/frame_timeline.txt
