#!/bin/bash
# Interleaved A/B of the frame rows: step-s records over every computed site
# (SQ_LIB variant, the build before) vs own rows/planes only (HEAD).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_fown_ab}
mkdir -p $O
for r in 1 2 3; do
  for v in allrec own; do  # allrec: the build before the change under test
    lib=stochquant_amd/lib/libstochquant.so; [ $v = allrec ] && lib=stochquant_amd/lib/variants/libstochquant_allrec.so
    SQ_LIB=$lib timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f_${v}_$r.log 2>&1 || { cat $O/rows_f_${v}_$r.log; exit 3; }
    python3 -c "
import json
for l in open('$O/rows_f_${v}_$r.log'):
    if l.startswith('{') and 'f1' in l:
        d=json.loads(l); print('$v round $r raw', d['raw_steps_us'], 'batch', d['batch_frame_us'], 'frame', d['frame_us'])
"
  done
done
