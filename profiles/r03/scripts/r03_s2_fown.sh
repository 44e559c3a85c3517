#!/bin/bash
# Frame records over owned rows/planes only: phi4 + P2P GPU tests, then the frame rows twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_fown}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f_$r.log 2>&1 || { cat $O/rows_f_$r.log; exit 3; }
  grep f1 $O/rows_f_$r.log
done
