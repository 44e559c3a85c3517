#!/bin/bash
# Round 6 call 8: C1 (the 32,768-site QM1D chain) A/B -- this build (leader
# word by step parity, addressed arithmetically) against the round-5 grid
# kernel (one leader word), interleaved three times; the QM1D GPU tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c8}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qm1d.py > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_new_$r.log 2>&1 || { tail -5 $O/c1_new_$r.log; exit 3; }
  SQ_LIB=stochquant_amd/lib/variants/libstochquant_r5qm1d.so timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 \
    > $O/c1_r5_$r.log 2>&1 || { tail -5 $O/c1_r5_$r.log; exit 4; }
  echo "new $(grep -o '"ms_per_frame": [0-9.]*' $O/c1_new_$r.log)  r5 $(grep -o '"ms_per_frame": [0-9.]*' $O/c1_r5_$r.log)"
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 5; }
python3 -c "
import json
d = json.loads([l for l in open('$O/bench_driver.log') if l.startswith('{')][-1])
print('%.4e' % d['value'], d['oracle_check'], d['oracle_check_noise'], 'c1 %.3e' % d['c1_qm1d']['value'],
      'frames', d['frames_256']['overhead'], 'slab', d['slab_1gpu']['rccl'].get('ratio_to_single'), d['slab_1gpu']['p2p'].get('ratio_to_single'))
"
