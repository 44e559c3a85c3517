#!/bin/bash
# Round-4 call 2: K=20 region-overhead diagnosis, RCCL CTA cap sweep on the
# one-GPU slab path (self-exchange), then rocprofv3 kernel-trace variants of
# the driver command to locate round 4's exit-time profiler crash (the likely
# culprit runs last: a crash ends the call).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c2}
mkdir -p $O
timeout -k 10 200 python3 scripts/diag_region.py > $O/region.log 2>&1 || { tail $O/region.log; exit 2; }
tail -1 $O/region.log
S="--comm rccl --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for r in 1 2; do for m in 0 1 2 4 8 b; do
  if [ $m = b ]; then E="SQ_RCCL_BLOCKING=1"; else E="SQ_RCCL_MAX_CTAS=$m"; fi
  env $E timeout -k 10 180 python3 bench.py $S > $O/slab_${m}_$r.log 2>&1 || { tail $O/slab_${m}_$r.log; exit 3; }
  echo "ctas=$m run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/slab_${m}_$r.log)"
done; done
B="bench.py --steps 20 --warmup 5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pA -o run --output-format csv -- python3 $B --no-cpu-baseline --no-c1 > $O/pA.log 2>&1 || { grep -v '^    @' $O/pA.log | tail -5; exit 4; }
echo "pA ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pB -o run --output-format csv -- python3 $B --no-cpu-baseline > $O/pB.log 2>&1 || { grep -v '^    @' $O/pB.log | tail -5; exit 5; }
echo "pB ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pC -o run --output-format csv -- python3 $B --no-c1 > $O/pC.log 2>&1 || { grep -v '^    @' $O/pC.log | tail -5; exit 6; }
echo "pC ok"
find $O -name '*kernel_trace.csv' -delete
