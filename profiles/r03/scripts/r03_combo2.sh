#!/bin/bash
# QM1D hoist tests + timings, frame-code bisection, fused-kernel A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_c2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_qm1d.py tests/test_gpu_tauhost.py tests/test_gpu_selftest.py -x -q --timeout 120 --timeout-method thread > $O/qm1d_tests.log 2>&1; echo "qm1d tests rc=$?"; tail -3 $O/qm1d_tests.log
timeout -k 10 300 python -u scripts/bench_qm1d.py --ordering jacobi --no-cpu --frames 5 > $O/qm1d_bench.log 2>&1; echo "qm1d bench rc=$?"; cat $O/qm1d_bench.log | cut -c1-200
VARS="main empty norec nobmx noscan" OUT=r03_bisect bash scripts/r03_dpp_variants.sh
bash scripts/r03_ab_only.sh
