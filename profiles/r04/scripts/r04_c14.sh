#!/bin/bash
# Round-4 calls 14-15: C1 grid kernel A/B/C on one box after the QM1D GPU
# tests of the main build.  Call 14: base (round 3's step), cur (own sites in
# registers + shared-divisor quotients), new (cur + acquire-only fence after
# the grid barrier).  Call 15: base, udiv (base + fence + shared-divisor
# quotients only), new (base + the acquire-only fence).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c14}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py tests/test_gpu_tauhost.py \
  > $O/qm1d_tests.log 2>&1 || { tail -30 $O/qm1d_tests.log; exit 1; }
tail -1 $O/qm1d_tests.log
for r in 1 2 3; do for v in base udiv new; do
  if [ $v = new ]; then unset SQ_LIB; else export SQ_LIB=stochquant_amd/lib/ab/libstochquant_$v.so; fi
  timeout -k 10 120 python3 -u scripts/bench_c1.py > $O/c1_${v}_$r.log 2>&1 || { tail $O/c1_${v}_$r.log; exit 2; }
  echo "$v run=$r $(tail -1 $O/c1_${v}_$r.log)"
done; done
