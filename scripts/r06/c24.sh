#!/bin/bash
# Round 6 call 24: the P2P exchange in order on the interior stream
# (SQ_XCHG_ON_A=1), with and without the kernel-staged slot: the P2P suite,
# then the interleaved slab A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c24}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py > $O/tests_p2p.log 2>&1 || { tail -40 $O/tests_p2p.log; exit 2; }
tail -1 $O/tests_p2p.log
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 9 p2p:p2p p2p_kst_k0:p2p:SQ_P2P_KSTAGE=1,SQ_CORE_PAIRS=0 \
  p2p_a:p2p:SQ_XCHG_ON_A=1 p2p_a_kst:p2p:SQ_XCHG_ON_A=1,SQ_P2P_KSTAGE=1 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -1
