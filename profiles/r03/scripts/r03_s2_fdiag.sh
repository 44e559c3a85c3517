#!/bin/bash
# Diagnostic only (wrong records, frames stay stable): where a 256^3 frame
# launch's extra time goes -- HEAD vs no per-site records vs no flush.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_fdiag}
mkdir -p $O
for r in 1 2; do
  for v in head norec noflush; do
    lib=stochquant_amd/lib/libstochquant.so; [ $v != head ] && lib=stochquant_amd/lib/variants/libstochquant_$v.so
    SQ_LIB=$lib timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f_${v}_$r.log 2>&1 || { cat $O/rows_f_${v}_$r.log; exit 3; }
    python3 -c "
import json
for l in open('$O/rows_f_${v}_$r.log'):
    if l.startswith('{') and 'f1' in l:
        d=json.loads(l); print('$v round $r raw', d['raw_steps_us'], 'batch', d['batch_frame_us'], 'frame', d['frame_us'])
"
  done
done
