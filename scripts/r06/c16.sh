#!/bin/bash
# Round 6 call 16: the frame records' cheaper first entry per wave -- the
# frame / stability GPU tests, then the frames diagnostic against the
# previous build (SQ_LIB), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py \
  -k "frame or stab or rollback or guard or checkpoint or snapshot" tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_new_$r.log 2>&1 || { tail -20 $O/frames_new_$r.log; exit 3; }
  SQ_LIB=stochquant_amd/lib/variants/libstochquant_prev.so timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_prev_$r.log 2>&1 \
    || { tail -20 $O/frames_prev_$r.log; exit 4; }
  for v in new prev; do
    echo "$v run $r: $(grep -v '^/opt' $O/frames_${v}_$r.log | python3 -c 'import sys,json; print([(json.loads(l)["way"], round(json.loads(l)["overhead"],4)) for l in sys.stdin if l.startswith("{")])')"
  done
done
