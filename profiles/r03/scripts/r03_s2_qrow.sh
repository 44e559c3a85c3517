#!/bin/bash
# Row-prefetch fused kernel (SQ_TB2_QROW=1): bitwise phi4 tests with it forced,
# then an interleaved A/B of the 256^3 bench line (round-2 kernel, the queue
# kernel capped at 80 VGPRs, the uncapped build as an SQ_LIB variant).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_qrow}
mkdir -p $O
SQ_TB2_QROW=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py > $O/tests_qrow.log 2>&1 || { tail -30 $O/tests_qrow.log; exit 2; }
tail -1 $O/tests_qrow.log
for r in 1 2; do
  for v in base q80 q89; do
    lib=stochquant_amd/lib/libstochquant.so; q=1
    [ $v = base ] && q=0
    [ $v = q89 ] && lib=stochquant_amd/lib/variants/libstochquant_q89.so
    SQ_LIB=$lib SQ_TB2_QROW=$q timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-c3 --no-check > $O/b_${v}_$r.log 2>&1 || { tail $O/b_${v}_$r.log; exit 3; }
    python3 -c "
import json
for l in open('$O/b_${v}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$v round $r', round(d['ms_per_step']*1e3,3),'us/step wall', r['avg_step_us'], 'kernel', 'busy', r.get('busy_fraction'))
"
  done
done
