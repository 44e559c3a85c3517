#!/bin/bash
# Round 6 call 13: the P2P exchange with one two-range copy launch for the
# staging and one for both pulls -- P2P / slab GPU tests, the slab A/B, and
# the N = 8 rehearsal on one GPU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c13}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_p2p.py \
  "tests/test_gpu_phi4.py::test_core_pairs_ahead_of_the_exchange_bitwise" "tests/test_gpu_phi4.py::test_full_size_256_rccl_slab_fused_vs_oracle" "tests/test_gpu_phi4.py::test_gate_timeout_is_sticky" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
timeout -k 10 300 python3 scripts/r06/slab_ab.py 1000 7 rccl:rccl p2p:p2p p2p_streamops:p2p:SQ_P2P_STREAMOPS=1 > $O/slab_ab.log 2>&1 || { tail -20 $O/slab_ab.log; exit 3; }
python3 -c "
import json
d = json.loads([l for l in open('$O/slab_ab.log') if l.startswith('{')][-1])
for n, v in d['contexts'].items(): print(n, v['median_us'], v['ratio'], v['min_us'])
"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p2p -o run -- python3 scripts/r06/slab_trace.py p2p 320 \
  > $O/trace_p2p.log 2>&1 || { tail -20 $O/trace_p2p.log; exit 4; }
timeout -k 10 600 python3 bench.py --gpus 8 --same-device --steps 20 --warmup 5 --no-c5 > $O/bench_n8.log 2>&1 \
  || { tail -20 $O/bench_n8.log; exit 5; }
python3 -c "
import json
d = json.loads([l for l in open('$O/bench_n8.log') if l.startswith('{')][-1])
print({k: d.get(k) for k in ('n_gpus', 'multi_rank_check', 'oracle_check', 'oracle_check_noise', 'error')})
"
