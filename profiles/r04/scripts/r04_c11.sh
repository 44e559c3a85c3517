#!/bin/bash
# Round-4 call 11: the frame kernels' record flush without the 64-bit DPP scans
# (only lanes holding the wave's maximum post their key) -- frame/record tests
# against the oracle, then the 20-step frame rows against the previous build
# (stochquant_amd/lib/ab/libstochquant_base.so via SQ_LIB), interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c11}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_fuzz.py \
  -k "frame or stab or guard or snapshot or checkpoint or record" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 1; }
tail -1 $O/frame_tests.log
BASE=stochquant_amd/lib/ab/libstochquant_base.so
for r in 1 2 3 4; do for v in base new; do
  if [ $v = base ]; then export SQ_LIB=$BASE; else unset SQ_LIB; fi
  timeout -k 10 200 python3 -u scripts/bench_rows_f.py > $O/rows_f_${v}_$r.log 2>&1 || { tail $O/rows_f_${v}_$r.log; exit 2; }
  echo "frames $v run=$r $(grep -h 'f1' $O/rows_f_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["raw_steps_us"], d["batch_frame_us"], d["frame_us"])')"
done; done
unset SQ_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ftr -o run --output-format csv -- python3 -u scripts/bench_rows_f.py > $O/rows_f_trace.log 2>&1 || { tail $O/rows_f_trace.log; exit 3; }
f=$(find $O/ftr -name '*kernel_trace.csv' | head -1)
python3 scripts/frame_timeline.py "$f" > $O/frame_timeline.txt 2>&1; cat $O/frame_timeline.txt
cp $(find $O/ftr -name '*kernel_stats.csv' | head -1) $O/rows_f_kernel_stats.csv
find $O/ftr -name '*kernel_trace.csv' -delete
# EDGES_DONE as the stop event of the pair before it (SQ_EDGES_STOPEV)
[ -n "$SKIP_SLAB" ] && exit 0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py \
  -k "core_pairs_ahead" > $O/slab_tests.log 2>&1 || { tail -30 $O/slab_tests.log; exit 4; }
tail -1 $O/slab_tests.log
S="--steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-c1 --no-check"
for r in 1 2; do for t in rccl p2p; do for v in 0 1; do
  SQ_EDGES_STOPEV=$v timeout -k 10 180 python3 bench.py --comm $t $S > $O/slab_${t}_ev${v}_$r.log 2>&1 || { tail $O/slab_${t}_ev${v}_$r.log; exit 5; }
  echo "$t stopev=$v run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/slab_${t}_ev${v}_$r.log)"
done; done; done
