#!/bin/bash
# Round 6 call 7: P2P with two linear staging copies, edges-first on/off, and
# the price of the exchange wait (SQ_DIAG_NO_XWAIT: no wait, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c7}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_p2p.py > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 300 python3 scripts/r06/slab_ab.py 1000 7 rccl:rccl rccl_nowait:rccl:SQ_DIAG_NO_XWAIT=1 p2p:p2p \
  p2p_ef0:p2p:SQ_EDGE_FIRST=0 p2p_nowait:p2p:SQ_DIAG_NO_XWAIT=1 rccl_ef1:rccl:SQ_EDGE_FIRST=1 > $O/slab_ab.log 2>&1 \
  || { tail -20 $O/slab_ab.log; exit 3; }
python3 -c "
import json
d = json.loads([l for l in open('$O/slab_ab.log') if l.startswith('{')][-1])
for n, v in d['contexts'].items(): print(n, v['median_us'], v['ratio'], v['min_us'])
"
