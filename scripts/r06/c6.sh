#!/bin/bash
# Round 6 call 6: the retightened tolerance tests, an interleaved A/B of the
# slab contexts (every context open, medians of 7 rounds), and a kernel trace
# of the new P2P exchange chain.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c6}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_phi4.py::test_stability_rule_quiet_on_stable_frames" "tests/test_gpu_qm1d.py::test_frame_within_tolerance" \
  > $O/t_tol.log 2>&1 || { tail -30 $O/t_tol.log; exit 2; }
tail -1 $O/t_tol.log
timeout -k 10 300 python3 scripts/r06/slab_ab.py 1000 7 rccl:rccl rccl_prio0:rccl:SQ_XCHG_PRIO=0 rccl_g12:rccl:SQ_GHOST=12 \
  rccl_stopev:rccl:SQ_EDGES_STOPEV=1 p2p:p2p p2p_prio0:p2p:SQ_XCHG_PRIO=0 p2p_g12:p2p:SQ_GHOST=12 > $O/slab_ab.log 2>&1 \
  || { tail -20 $O/slab_ab.log; exit 3; }
python3 -c "
import json
d = json.loads([l for l in open('$O/slab_ab.log') if l.startswith('{')][-1])
for n, v in d['contexts'].items(): print(n, v['median_us'], v['ratio'], v['min_us'])
"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p2p -o run -- python3 scripts/r06/slab_trace.py p2p 320 \
  > $O/trace_p2p.log 2>&1 || { tail -20 $O/trace_p2p.log; exit 4; }
grep us/step $O/trace_p2p.log
