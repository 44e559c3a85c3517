#!/bin/bash
# Round 6 call 29: one rank's RCCL self-exchange in order -- each face as
# k RCCL sends / receives (SQ_RCCL_SPLIT) so RCCL can spread them; bitwise
# check first, then the interleaved A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c29}
mkdir -p $O
SQ_RCCL_SPLIT=4 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "rccl or exchange_on_interior" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 9 rccl:rccl rccl_s2:rccl:SQ_RCCL_SPLIT=2 rccl_s4:rccl:SQ_RCCL_SPLIT=4 rccl_s8:rccl:SQ_RCCL_SPLIT=8 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep '^{' $O/slab_ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); [print(k, v["ratio"], v["median_us"]) for k,v in d["contexts"].items()]'
