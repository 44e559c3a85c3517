#!/bin/bash
# Round 6 calls 4+5 in one: the P2P change's GPU tests first (c5.sh's tests),
# then the slab schedule sweep and frame variants (c4.sh), then the N = 8
# rehearsal on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/r06_c45
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  "tests/test_gpu_phi4.py::test_core_pairs_ahead_of_the_exchange_bitwise" "tests/test_gpu_phi4.py::test_gate_timeout_is_sticky" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 400 python3 scripts/r06/slab_sweep.py 1000 > $O/slab_sweep.log 2>&1 || { tail -20 $O/slab_sweep.log; exit 3; }
grep '"rep": 1' $O/slab_sweep.log
for v in "SQ_FRAME_FOLD=0" "SQ_FRAME_TRI=0"; do
  env $v timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_$v.log 2>&1 || { tail -20 $O/frames_$v.log; exit 4; }
  echo $v; grep alternate $O/frames_$v.log
done
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 > $O/bench_n8.log 2>&1 \
  || { tail -20 $O/bench_n8.log; exit 5; }
python3 - <<PY
import json
d = json.loads([l for l in open("$O/bench_n8.log") if l.startswith("{")][-1])
print({k: d.get(k) for k in ("value", "n_gpus", "ms_per_step", "multi_rank_check", "oracle_check", "oracle_check_noise", "error")})
c5 = d.get("c5_1024", {})
print("c5", {k: c5.get(k) for k in ("value", "multi_rank_check", "oracle_check", "oracle_check_noise", "error")})
PY
