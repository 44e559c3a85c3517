#!/bin/bash
# Round 5, call 14: per-block records replace the leader/instability atomics and
# the dependent load of X' at E: every QM1D / serial / tauhost GPU test, C1 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c14}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_qm1d.py tests/test_gpu_qm1d_serial.py tests/test_gpu_tauhost.py > $O/qm1d.log 2>&1 || { tail -30 $O/qm1d.log; exit 3; }
tail -1 $O/qm1d.log
for r in 1 2; do
  timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_$r.log 2>&1 || { tail -5 $O/c1_$r.log; exit 4; }
  echo "c1 default run=$r $(grep '^{' $O/c1_$r.log)"
done
