#!/bin/bash
# Two-step kernel band height A/B (SQ_TB2_ROWS 8 vs 14) at 256^3, interleaved,
# (Measured and not adopted: the 14-row code was removed after this A/B; profiles/r02/ab/rows14/.)
# after the bitwise fused-kernel tests under 14-row bands.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/rows_ab
mkdir -p $O
SQ_TB2_ROWS=14 timeout -k 10 400 python -u -m pytest tests/test_gpu_phi4.py tests/test_gpu_fuzz.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/tests_rows14.log 2>&1 || { tail -30 $O/tests_rows14.log; exit 1; }
tail -1 $O/tests_rows14.log
for rnd in 1 2 3; do
  for r in 8 14; do
    echo "rows $r round $rnd: $(SQ_TB2_ROWS=$r timeout -k 10 100 python3 scripts/sweep_tb2.py --shape ${SHAPE:-256x256x256} \
       --steps 1000 --rounds 2 --variants fuse1,wpe6,bpc2 2>&1 | grep 'us ' | tail -1)"
  done
done
