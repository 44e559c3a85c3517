#!/bin/bash
# Round 6 call 20: the kernel-staged P2P exchange (SQ_P2P_KSTAGE=1): the P2P
# GPU suite (kstage cases included), a kernel trace of the P2P self-exchange
# with it (the stage kernel launched, no staging copy), then the interleaved
# slab A/B: P2P with and without it, RCCL.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c20}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py > $O/tests_p2p.log 2>&1 || { tail -40 $O/tests_p2p.log; exit 2; }
tail -1 $O/tests_p2p.log
export TMPDIR=/tmp
SQ_P2P_KSTAGE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/tr_kst -o run -- python3 scripts/r06/slab_trace.py p2p 320 > $O/tr_kst.log 2>&1 || { tail -20 $O/tr_kst.log; exit 3; }
find $O/tr_kst -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-4 {} | head -12
timeout -k 10 400 python3 -u scripts/r06/slab_ab.py 1000 7 p2p:p2p p2p_kst:p2p:SQ_P2P_KSTAGE=1 rccl:rccl > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -8
