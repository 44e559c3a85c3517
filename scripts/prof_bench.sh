#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench command (profiles/<round>/).
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o run --output-format csv \
   -- python3 "$R/bench.py" --no-cpu-baseline
find "$R/gpurun_out/prof_bench" -name "*kernel_stats.csv" -exec cat {} \;
