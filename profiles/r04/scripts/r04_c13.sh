#!/bin/bash
# Round-4 call 13: the QM1D grid kernel (C1) with its own sites kept in
# registers and the step's quotients by the shared-divisor form -- the QM1D
# and tauhost GPU tests (bitwise vs the one-CU kernel and the oracle), then the
# driver's invocation twice for the c1_qm1d sub-record.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c13}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py tests/test_gpu_tauhost.py tests/test_gpu_fuzz.py \
  > $O/qm1d_tests.log 2>&1 || { tail -30 $O/qm1d_tests.log; exit 1; }
tail -1 $O/qm1d_tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail $O/bench_driver_$r.log; exit 2; }
  python3 - $O/bench_driver_$r.log <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
c = d["c1_qm1d"]
print(d["value"], d["ms_per_step"], "| c1", c["value"], c["ms_per_frame"], c["kernel_ms_per_frame"], c["cpu_baseline"]["value"])
EOF
done
