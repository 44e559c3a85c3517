#!/bin/bash
# Round 6 call 25: the exchange in order on the interior stream for RCCL too:
# its bitwise tests (RCCL / P2P, kstage, G 4 / 16), the P2P suite, then the
# slab A/B of RCCL and P2P with and without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c25}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py \
  -k "exchange_on_interior or core_pairs_ahead or rccl" tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 9 rccl:rccl rccl_a:rccl:SQ_XCHG_ON_A=1 p2p:p2p \
  p2p_a_kst:p2p:SQ_XCHG_ON_A=1,SQ_P2P_KSTAGE=1 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -1
