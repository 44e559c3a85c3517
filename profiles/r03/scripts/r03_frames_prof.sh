#!/bin/bash
# Kernel times of frame launches vs raw steps (256^3, 20-step frames).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_fprof}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_rows_f.py --reps 20 > $O/rows_f.log 2>&1 || { tail -20 $O/rows_f.log; exit 2; }
cat $O/rows_f.log | grep f1
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null || ls $O/prof/run_kernel_stats.csv)
head -20 $f
