#!/bin/bash
# Round 6 call 21: the kernel-staged P2P exchange with the block start's other
# hop changed too: the rims gated in-kernel on the exchange (SQ_SLAB_GATE=1),
# or no core / rim split (SQ_CORE_PAIRS=0); interleaved against plain P2P.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c21}
mkdir -p $O
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 7 p2p:p2p p2p_kst:p2p:SQ_P2P_KSTAGE=1 \
  p2p_kst_gate:p2p:SQ_P2P_KSTAGE=1,SQ_SLAB_GATE=1 p2p_kst_k0:p2p:SQ_P2P_KSTAGE=1,SQ_CORE_PAIRS=0 \
  p2p_gate:p2p:SQ_SLAB_GATE=1 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -3
