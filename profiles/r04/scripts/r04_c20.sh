#!/bin/bash
# Round-4 call 20: the default bench line (no flags: 2000 timed steps, c3_512,
# c1_qm1d, CPU baselines) and the 1024^3 lattice (C5's per-node lattice on one GPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c20}
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench_default.log 2>&1 || { tail $O/bench_default.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e-]*\|"frac": [0-9.]*\|"clock_MHz_measured": [0-9.]*' $O/bench_default.log | head -12
timeout -k 10 300 python3 bench.py --size 1024 --steps 200 --warmup 20 --no-c3 --no-c1 --no-cpu-baseline > $O/bench_1024.log 2>&1 || { tail $O/bench_1024.log; exit 2; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e-]*\|"clock_MHz_measured": [0-9.]*\|"busy_fraction": [0-9.]*' $O/bench_1024.log | head -6
