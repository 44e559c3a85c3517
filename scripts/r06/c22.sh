#!/bin/bash
# Round 6 call 22: P2P with / without the kernel-staged exchange, 15
# interleaved rounds; and a kernel trace of the pathological K = 0 + kstage case.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c22}
mkdir -p $O
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 15 p2p:p2p p2p_kst:p2p:SQ_P2P_KSTAGE=1 rccl:rccl > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -1
export TMPDIR=/tmp
SQ_CORE_PAIRS=0 SQ_P2P_KSTAGE=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_k0 -o run -- python3 scripts/r06/slab_trace.py p2p 160 > $O/tr_k0.log 2>&1 || { tail -20 $O/tr_k0.log; exit 3; }
tail -2 $O/tr_k0.log
