#!/bin/bash
# Round 6 call 26: one rank's self-exchange in order on stream A by default
# (P2P with the staged last pair): the phi4 / P2P / march GPU suites, the slab
# A/B of the new defaults against the overlapped form, then the driver's bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c26}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_p2p.py tests/test_gpu_run.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 9 rccl:rccl rccl_b:rccl:SQ_XCHG_ON_A=0 p2p:p2p p2p_b:p2p:SQ_XCHG_ON_A=0 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep -v "amdgpu.ids" $O/slab_ab.log | tail -1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 5; }
grep '^{"metric"' $O/bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["oracle_check"], d.get("oracle_check_noise"), json.dumps(d.get("slab_1gpu"))[:900])'
