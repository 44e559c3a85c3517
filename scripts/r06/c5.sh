#!/bin/bash
# Round 6 call 5: P2P exchange with double-buffered staged copies and no
# per-exchange acknowledgements -- the P2P / slab GPU tests (2-8 rank
# processes, bitwise vs the single slab), the slab ratios, and the N = 8
# rehearsal on one GPU (P2P fallback) with every check.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  "tests/test_gpu_phi4.py::test_core_pairs_ahead_of_the_exchange_bitwise" "tests/test_gpu_phi4.py::test_gate_timeout_is_sticky" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 300 python3 scripts/r06/slab_sweep.py 1000 p2ponly > $O/slab_p2p.log 2>&1 || { tail -20 $O/slab_p2p.log; exit 3; }
cat $O/slab_p2p.log
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 > $O/bench_n8.log 2>&1 \
  || { tail -20 $O/bench_n8.log; exit 4; }
python3 - <<PY
import json
d = json.loads([l for l in open("$O/bench_n8.log") if l.startswith("{")][-1])
print({k: d.get(k) for k in ("value", "n_gpus", "ms_per_step", "multi_rank_check", "oracle_check", "oracle_check_noise", "error")})
c5 = d.get("c5_1024", {})
print("c5", {k: c5.get(k) for k in ("value", "multi_rank_check", "oracle_check", "oracle_check_noise", "error")})
PY
