#!/bin/bash
# Round-4 call 8: the neighbour-sync fused kernel (SQ_TB2_SYNC=p2p: row waves
# wait for their two neighbours' progress words, no block barrier per plane)
# against the barrier kernel: bitwise test, then interleaved 256^3 benches and
# one kernel-stats pass each.  Stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c8}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_phi4.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "neighbour_sync or frame_launches_equal or loopback_decomposition or run_frames" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for r in 1 2 3; do for s in barrier p2p; do
  SQ_TB2_SYNC=$s timeout -k 10 180 python3 bench.py $B > $O/b_${s}_$r.log 2>&1 || { tail $O/b_${s}_$r.log; exit 2; }
  echo "$s run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${s}_$r.log)"
done; done
for s in barrier p2p; do
  SQ_TB2_SYNC=$s timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/st_$s -o run --output-format csv -- python3 bench.py --steps 200 --warmup 50 --settle-ms 300 --no-cpu-baseline --no-c3 --no-c1 --no-check > $O/st_$s.log 2>&1 || { tail $O/st_$s.log; exit 3; }
  f=$(find $O/st_$s -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_$s.csv
  find $O/st_$s -name '*kernel_trace.csv' -delete
  echo "$s $(grep phi4_tb2 $O/kernel_stats_$s.csv | head -2 | cut -c1-200)"
done
for r in 1 2; do for s in barrier p2p; do
  SQ_TB2_SYNC=$s timeout -k 10 200 python3 -u scripts/bench_rows_f.py > $O/rows_f_${s}_$r.log 2>&1 || { tail $O/rows_f_${s}_$r.log; exit 4; }
  echo "frames $s run=$r $(grep -h 'f1' $O/rows_f_${s}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["raw_steps_us"], d["batch_frame_us"], d["frame_us"])')"
done; done
