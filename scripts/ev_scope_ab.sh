#!/bin/bash
# Interleaved A/B of the slab path's event fence scope (SQ_EV_SCOPE), RCCL
# self-exchange at 256^3, plus the bitwise slab tests under the candidate.
# (The SQ_EV_SCOPE knob existed only for this A/B; it was removed after it: no gain.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/ev_scope
mkdir -p $O
SQ_EV_SCOPE=device timeout -k 10 300 python -u -m pytest tests/test_gpu_phi4.py tests/test_gpu_p2p.py -m gpu -x -q \
  -k "rccl or slab or deep_halo or core_pairs or p2p" --timeout 120 --timeout-method thread > $O/tests_device.log 2>&1 || { tail -20 $O/tests_device.log; exit 1; }
tail -1 $O/tests_device.log
for rnd in 1 2 3; do
  for m in default device nofence; do
    SQ_EV_SCOPE=$m timeout -k 10 120 python bench.py --comm ${COMM:-rccl} --steps 1600 --warmup 200 --settle-ms 500 \
      --no-cpu-baseline --no-profile-events > $O/${m}_$rnd.log 2>&1 || exit 2
    echo "$m round $rnd: $(grep -o '"ms_per_step": [0-9.]*' $O/${m}_$rnd.log)"
  done
done
