#!/bin/bash
# QM1D tests + Jacobi frame timings (shared-divisor division), then frame vs raw kernel times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py tests/test_gpu_qm1d_serial.py tests/test_gpu_tauhost.py > $O/qm1d_tests.log 2>&1 || { tail -30 $O/qm1d_tests.log; exit 2; }
tail -1 $O/qm1d_tests.log
timeout -k 10 300 python -u scripts/bench_qm1d.py --ordering jacobi --no-cpu > $O/qm1d_bench.log 2>&1 || { tail $O/qm1d_bench.log; exit 3; }
cat $O/qm1d_bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/bench_rows_f.py --reps 20 > $O/rows_f_prof.log 2>&1 || { tail -20 $O/rows_f_prof.log; exit 4; }
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null || ls $O/prof/run_kernel_stats.csv)
cut -c1-200 $f | head -12
