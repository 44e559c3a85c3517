#!/bin/bash
# Round-4 call 7: (1) the profile of the driver's exact bench invocation
# (profiles/r04/), (2) the full GPU suite + smoke, (3) slab path: gated pair 0
# on/off and the exchange-overlap block target, with kernel timelines.
# A failing test does not stop the call; a fault, abort, crash or time limit does.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c7}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
bash scripts/r04_driver_prof.sh ${1:-r04_c7}/prof; rc=$?; echo "driver_prof rc=$rc"; fatal $rc prof
[ $rc -eq 0 ] || exit $rc
bash scripts/r04_suite.sh ${1:-r04_c7}/suite; rc=$?; echo "suite rc=$rc"; fatal $rc suite
S="--comm rccl --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for g in 0 1; do
  SQ_SLAB_GATE=$g timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_g$g -o run --output-format csv -- python3 bench.py --comm rccl --steps 200 --warmup 50 --settle-ms 300 --no-cpu-baseline --no-c3 --no-c1 --no-check > $O/tl_g$g.log 2>&1; rc=$?; fatal $rc tl; [ $rc -eq 0 ] || { tail $O/tl_g$g.log; exit 2; }
  python3 scripts/slab_timeline.py $(find $O/tl_g$g -name '*kernel_trace.csv' | head -1) 40 > $O/timeline_g$g.txt
  find $O/tl_g$g -name '*kernel_trace.csv' -delete
done
for r in 1 2; do for cfg in "0 416" "1 416" "1 352" "1 480"; do
  set -- $cfg
  SQ_SLAB_GATE=$1 SQ_XCHG_BLOCKS=$2 timeout -k 10 180 python3 bench.py $S > $O/rccl_g$1_$2_$r.log 2>&1; rc=$?; fatal $rc sweep; [ $rc -eq 0 ] || { tail $O/rccl_g$1_$2_$r.log; exit 3; }
  echo "rccl gate=$1 xb=$2 run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/rccl_g$1_$2_$r.log)"
done; done
for r in 1 2; do for g in 0 1; do
  SQ_SLAB_GATE=$g timeout -k 10 180 python3 bench.py --comm p2p --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check > $O/p2p_g${g}_$r.log 2>&1; rc=$?; fatal $rc p2p; [ $rc -eq 0 ] || { tail $O/p2p_g${g}_$r.log; exit 3; }
  echo "p2p gate=$g run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/p2p_g${g}_$r.log)"
done; done
# (4) the neighbour-sync A/B (scripts/r04_c8.sh) when the call has time left
if [ $SECONDS -lt 650 ]; then bash scripts/r04_c8.sh ${1:-r04_c7}/p2sync; rc=$?; echo "p2sync rc=$rc"; fi
