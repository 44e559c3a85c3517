#!/bin/bash
# Round evidence on one GPU: the GPU test suite, the default bench line, the
# rocprofv3 kernel-trace summary of the same command, and the PMC traffic passes.
#   bash scripts/gpu_evidence.sh TAG
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { cat gpurun_out/bench_$TAG.log; exit 1; }
grep '^{' gpurun_out/bench_$TAG.log
bash scripts/prof_bench.sh > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
STEPS=30 bash scripts/pmc_run.sh 256 $TAG > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
tail -1 gpurun_out/pmc_$TAG.log
