#!/bin/bash
# Round 6 call 23: the K = 0 + kstage slowdown seen in c21's A/B (2.77x) --
# alone with the single slab, then traced inside slab_ab.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c23}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/r06/slab_ab.py 1000 3 p2p_kst_k0:p2p:SQ_P2P_KSTAGE=1,SQ_CORE_PAIRS=0 p2p_k0:p2p:SQ_CORE_PAIRS=0 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_ab -o run -- python3 scripts/r06/slab_ab.py 200 2 p2p_kst_k0:p2p:SQ_P2P_KSTAGE=1,SQ_CORE_PAIRS=0 > $O/tr_ab.log 2>&1 || { tail -20 $O/tr_ab.log; exit 3; }
grep -v "amdgpu.ids\|rocprofv3\|^W" $O/tr_ab.log | tail -2
