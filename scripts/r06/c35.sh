#!/bin/bash
# Round 6 call 35: the block-end flush without its global atomics (noatomic) against no flush and the build itself; was call 34: where the frame launch's extra time goes -- diagnostic
# builds (results wrong, timing only): no M / D record work (norec), no
# per-float4 record work at all (nosites), no block-end flush (noflush),
# against the build itself, two interleaved rounds of scripts/r06/frames_diag.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c35}
mkdir -p $O
for r in 1 2 3; do
  for v in base noflush noatomic; do
    if [ $v = base ]; then unset SQ_LIB; else export SQ_LIB=stochquant_amd/lib/variants/libstochquant_$v.so; fi
    timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_${v}_$r.log 2>&1 || { tail -20 $O/frames_${v}_$r.log; exit 3; }
    echo "$v run $r: $(grep -v '^/opt' $O/frames_${v}_$r.log | python3 -c 'import sys,json; print([(json.loads(l)["way"], round(json.loads(l)["overhead"],4), round(json.loads(l).get("us_per_frame",0),1)) for l in sys.stdin if l.startswith("{")])')"
  done
done
