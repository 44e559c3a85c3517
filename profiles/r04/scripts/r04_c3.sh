#!/bin/bash
# Round-4 call 3: host-wait schedule vs the K=20 region overhead; then the C1
# path under rocprofv3 with the plain (non-cooperative) grid launch, last.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py > $O/qm1d_tests.log 2>&1 || { tail -30 $O/qm1d_tests.log; exit 2; }
tail -1 $O/qm1d_tests.log
for r in 1 2; do for f in none spin yield block; do
  timeout -k 10 120 python3 scripts/diag_region.py --flags $f --reps 30 > $O/region_${f}_$r.log 2>&1 || { tail $O/region_${f}_$r.log; exit 3; }
  tail -1 $O/region_${f}_$r.log
done; done
B="bench.py --steps 20 --warmup 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pB -o run --output-format csv -- python3 $B --no-cpu-baseline > $O/pB.log 2>&1 || { grep -v '^    @' $O/pB.log | tail -5; exit 5; }
echo "pB ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pC -o run --output-format csv -- python3 $B > $O/pC.log 2>&1 || { grep -v '^    @' $O/pC.log | tail -5; exit 6; }
echo "pC ok"
find $O -name '*kernel_trace.csv' -delete
