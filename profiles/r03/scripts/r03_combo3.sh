#!/bin/bash
# Full GPU suite, frames-vs-steps diag for both kernels, kernel A/B, golden slab digests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_c3
mkdir -p $O
timeout -k 10 300 python -u scripts/make_golden_slabs.py gpurun_out/golden_slabs.json > $O/golden.log 2>&1; echo "golden rc=$?"; tail -3 $O/golden.log
cp gpurun_out/golden_slabs.json stochquant_amd/golden_slabs.json || exit 3
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -80; exit 1; }
REPS=10 VARS="main" OUT=r03_c3/diag bash scripts/r03_dpp_variants.sh || exit 2
bash scripts/r03_ab_only.sh r03_c3_ab
