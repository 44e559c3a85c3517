#!/bin/bash
# Round 6 call 37: the flush atomics XCD-local -- 256 slots per step, block b on XCD x posts into x's 32 (own cache lines), workgroup-scope atomics performed in that XCD's L2 (the kernel boundary publishes them) -- bitwise frame tests and frames_diag against the build, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c37}
mkdir -p $O
SQ_LIB=stochquant_amd/lib/variants/libstochquant_xccslots.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py \
  -k "frame or stab or rollback" tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in base xccslots; do
    if [ $v = base ]; then unset SQ_LIB; else export SQ_LIB=stochquant_amd/lib/variants/libstochquant_$v.so; fi
    timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_${v}_$r.log 2>&1 || { tail -20 $O/frames_${v}_$r.log; exit 3; }
    echo "$v run $r: $(grep -v '^/opt' $O/frames_${v}_$r.log | python3 -c 'import sys,json; print([(json.loads(l)["way"], round(json.loads(l)["overhead"],4)) for l in sys.stdin if l.startswith("{")])')"
  done
done
