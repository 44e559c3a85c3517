#!/bin/bash
# Round 6 call 15: what the EDGES_DONE dependency costs (SQ_DIAG_NO_EWAIT:
# no event, the exchange races the last pair -- timing only) and both waits
# removed, RCCL and P2P, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c15}
mkdir -p $O
timeout -k 10 300 python3 scripts/r06/slab_ab.py 1000 7 rccl:rccl rccl_noe:rccl:SQ_DIAG_NO_EWAIT=1 \
  rccl_none:rccl:SQ_DIAG_NO_EWAIT=1,SQ_DIAG_NO_XWAIT=1 p2p:p2p p2p_noe:p2p:SQ_DIAG_NO_EWAIT=1 \
  p2p_none:p2p:SQ_DIAG_NO_EWAIT=1,SQ_DIAG_NO_XWAIT=1 > $O/slab_ab.log 2>&1 || { tail -20 $O/slab_ab.log; exit 3; }
python3 -c "
import json
d = json.loads([l for l in open('$O/slab_ab.log') if l.startswith('{')][-1])
for n, v in d['contexts'].items(): print(n, v['median_us'], v['ratio'], v['min_us'])
"
