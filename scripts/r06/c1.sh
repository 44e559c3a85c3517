#!/bin/bash
# Round 6 call 1: the changed paths' GPU tests (sticky gate timeout, the QM1D
# grid kernel's parity-indexed leader word, 8 P2P rank processes), then the
# driver's N = 8 shape on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/${1:-r06_c1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_p2p.py tests/test_gpu_qm1d.py "tests/test_gpu_phi4.py::test_gate_timeout_is_sticky" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 > $O/bench_n8.log 2>&1 \
  || { tail -20 $O/bench_n8.log; exit 4; }
python3 - <<PY
import json
d = json.loads([l for l in open("$O/bench_n8.log") if l.startswith("{")][-1])
print({k: d.get(k) for k in ("value", "n_gpus", "ms_per_step", "multi_rank_check", "oracle_check", "transport_fallback", "error")})
c5 = d.get("c5_1024", {})
print("c5", {k: c5.get(k) for k in ("value", "multi_rank_check", "oracle_check", "error")})
PY
