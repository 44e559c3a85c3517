#!/bin/bash
# Slab-path GPU tests (phi4 + P2P ranks), then the one-GPU slab bench lines
# (RCCL and P2P self-exchange) at the new defaults.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_slab2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2; do
  for c in rccl p2p; do
    timeout -k 10 180 python bench.py --comm $c --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check > $O/b_${c}_$r.log 2>&1 || exit 3
    python3 -c "
import json
for l in open('$O/b_${c}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); c=d['config']; print('$c round $r', round(d['ms_per_step']*1e3,3),'us/step', c.get('ghost_depth'), c.get('block_schedule'))
"
  done
done
