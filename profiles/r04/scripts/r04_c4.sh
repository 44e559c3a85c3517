#!/bin/bash
# Round-4 call 4: slab-path launches beside an exchange aim at fewer blocks
# (SQ_XCHG_BLOCKS); the decomposition tests stay bitwise; A/B of the target on
# the one-GPU RCCL and P2P self-exchange, interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c4}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_p2p.py -k "rccl or loopback or deep_halo or ghost or uneven or core_pairs or p2p or c5" > $O/slab_tests.log 2>&1 || { tail -30 $O/slab_tests.log; exit 2; }
tail -1 $O/slab_tests.log
S="--steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for r in 1 2; do for comm in rccl p2p; do for xb in 512 496 480 448 416; do
  SQ_XCHG_BLOCKS=$xb timeout -k 10 180 python3 bench.py --comm $comm $S > $O/${comm}_${xb}_$r.log 2>&1 || { tail $O/${comm}_${xb}_$r.log; exit 3; }
  echo "$comm xb=$xb run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/${comm}_${xb}_$r.log)"
done; done; done
