#!/bin/bash
# Round-4 call 16: the multi-process bench paths on one GPU -- two ranks on
# GPU 0 with the default transport (RCCL refuses two ranks on one device, so
# this exercises the P2P fallback end to end) and with --comm p2p -- then the
# full GPU suite and smoke().
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c16}
mkdir -p $O
B="--gpus 2 --same-device --steps 200 --warmup 20 --no-c3 --no-c1 --rank-timeout 240"
timeout -k 10 300 python3 bench.py $B > $O/bench_2r_auto.log 2>&1; rc=$?
echo "auto rc=$rc"; grep -o '"value": [0-9.e+]*\|"parallelism": "[^"]*"\|"transport_fallback": [^,]*,\|"multi_rank_check": "[^"]*"\|"error": "[^"]*"' $O/bench_2r_auto.log | head -8
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py $B --comm p2p > $O/bench_2r_p2p.log 2>&1; rc=$?
echo "p2p rc=$rc"; grep -o '"value": [0-9.e+]*\|"parallelism": "[^"]*"\|"transport_fallback": [^,]*,\|"multi_rank_check": "[^"]*"' $O/bench_2r_p2p.log | head -8
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/r04_suite.sh ${1:-r04_c16}/suite
