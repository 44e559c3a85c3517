#!/bin/bash
# 256^3: the 8-waves-per-SIMD register budget (SQ_TB2_WPE_N=8, 63-64 VGPRs)
# with 2 or 3 blocks per CU, both fused kernels, vs the default; then the
# phi4 parity tests under the best-guess setting.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_wpe8}
mkdir -p $O
B="bench.py --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check"
for r in 1 2; do
  for cfg in "0 1 2" "0 8 2" "0 8 3" "1 8 2" "1 8 3"; do
    set -- $cfg
    SQ_TB2_PIPE=$1 SQ_TB2_WPE_N=$2 SQ_TB2_BLOCKS_PER_CU=$3 timeout -k 10 120 python $B > $O/b256_p$1_w$2_b$3_$r.log 2>&1 || exit 2
  done
done
for f in $O/b*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step', '%.3e'%d['value'], r['avg_launch_us'], r['kernel'][:60])
"; done
SQ_TB2_PIPE=1 SQ_TB2_WPE_N=8 SQ_TB2_BLOCKS_PER_CU=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py > $O/tests_p1_w8_b3.log 2>&1 || exit 3
SQ_TB2_PIPE=0 SQ_TB2_WPE_N=8 SQ_TB2_BLOCKS_PER_CU=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py > $O/tests_p0_w8_b3.log 2>&1 || exit 4
tail -2 $O/tests_*.log
