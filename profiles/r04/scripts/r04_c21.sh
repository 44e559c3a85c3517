#!/bin/bash
# Round-4 call 21: the driver's multi-GPU launch mode rehearsed on one GPU --
# torch.distributed.run with two ranks (no spawning parent), both on GPU 0
# (--same-device), default transport (RCCL refuses the shared device -> the
# ranks agree on the P2P fallback).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c21}
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --same-device --steps 20 --warmup 5 --no-c3 --no-c1 > $O/torchrun_2.log 2>&1; rc=$?
echo "rc=$rc"
grep '^{' $O/torchrun_2.log | cut -c1-600
