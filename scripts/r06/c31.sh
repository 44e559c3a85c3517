#!/bin/bash
# Round 6 call 31: the P2P destroy drain ordered after in-order pulls -- the
# P2P suite and the slab tests of the phi4 suite; then the driver's N = 8
# shape on one GPU (which schedule the timed pick takes).
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c31}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 --no-c3 --no-c1 > $O/bench_n8.log 2>&1 || { tail -20 $O/bench_n8.log; exit 3; }
grep '^{"metric"' $O/bench_n8.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["multi_rank_check"], d["oracle_check"], d.get("oracle_check_noise"), d.get("transport"), json.dumps(d.get("schedule", d.get("config",{}).get("schedule")))[:400])'
