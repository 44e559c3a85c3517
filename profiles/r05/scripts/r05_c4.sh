#!/bin/bash
# Round 5, call 4: the device hash field and the oracle protocol on it, the
# driver's bench command with the 1024^3 strong-scaling sub-record, and the
# two-rank P2P line on one GPU (c5 at N = 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c4}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_phi4.py -k "init_field_hash or oracle_protocol or oracle_check_full" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 3; }
timeout -k 10 400 python3 bench.py --gpus 2 --same-device --comm p2p --steps 20 --warmup 5 > $O/p2p_2ranks.log 2>&1 || { tail -20 $O/p2p_2ranks.log; exit 4; }
