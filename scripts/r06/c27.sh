#!/bin/bash
# Round 6 call 27: one rank's RCCL self-exchange in order on stream A -- does
# RCCL's channel count move it?  One process per setting (RCCL caches its
# parameters per process), each with its own single-slab baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c27}
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python3 -u scripts/r06/slab_ab.py 1000 5 rccl:rccl > $O/ab_$n.log 2>&1 || { tail -20 $O/ab_$n.log; return 1; }
  echo "$n: $(grep '^{' $O/ab_$n.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["contexts"]["rccl"]["ratio"], d["contexts"]["rccl"]["median_us"])')"
}
run default SQ_NONE=0 && \
run p2pch8 NCCL_NCHANNELS_PER_PEER=8 && run p2pch16 NCCL_MIN_P2P_NCHANNELS=16 NCCL_MAX_P2P_NCHANNELS=32 && run default2 SQ_NONE=0
