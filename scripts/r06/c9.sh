#!/bin/bash
# Round 6 call 9: the rim pair's chunk depth (SQ_TB2_MINZ 2 / 3 against the
# default 4) in the interleaved slab A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c9}
mkdir -p $O
timeout -k 10 300 python3 scripts/r06/slab_ab.py 1000 7 rccl:rccl rccl_z2:rccl:SQ_TB2_MINZ=2 rccl_z3:rccl:SQ_TB2_MINZ=3 \
  p2p:p2p p2p_z2:p2p:SQ_TB2_MINZ=2 > $O/slab_ab.log 2>&1 || { tail -20 $O/slab_ab.log; exit 3; }
python3 -c "
import json
d = json.loads([l for l in open('$O/slab_ab.log') if l.startswith('{')][-1])
for n, v in d['contexts'].items(): print(n, v['median_us'], v['ratio'], v['min_us'])
"
