#!/bin/bash
# Round 6 call 28: ghost depth for the in-order exchange on one GPU: G = 8 / 12
# against the default 16, RCCL and P2P, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c28}
mkdir -p $O
timeout -k 10 600 python3 -u scripts/r06/slab_ab.py 1000 9 rccl:rccl rccl_g8:rccl:SQ_GHOST=8 rccl_g12:rccl:SQ_GHOST=12 \
  p2p:p2p p2p_g8:p2p:SQ_GHOST=8 p2p_g12:p2p:SQ_GHOST=12 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep '^{' $O/slab_ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); [print(k, v["ratio"], v["median_us"]) for k,v in d["contexts"].items()]'
