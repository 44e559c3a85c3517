#!/bin/bash
# Kernel-level timing of the serial-order QM1D frame (rocprofv3 --kernel-trace --stats).
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_serial" -o run --output-format csv \
   -- python3 "$R/scripts/bench_qm1d.py" --ordering serial --frames 3
cat "$R"/gpurun_out/prof_serial/*/run_kernel_stats.csv 2>/dev/null || find "$R/gpurun_out/prof_serial" -name "*stats*" -exec cat {} \;
