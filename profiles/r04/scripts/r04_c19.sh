#!/bin/bash
# Round-4 call 19: the full GPU suite + smoke of the closing tree, then the
# driver's N = 1 invocation once.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c19}
mkdir -p $O
bash scripts/r04_suite.sh ${1:-r04_c19}/suite || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail $O/bench_driver.log; exit 4; }
grep -o '"value": [0-9.e+]*' $O/bench_driver.log | head -1
# the frame instance's VALU work after round 4's record trims, beside the raw instance
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $O/fpmc -o run --output-format csv -- python3 scripts/frames_only.py > $O/fpmc.log 2>&1 || { tail $O/fpmc.log; exit 5; }
python3 scripts/pmc_sq_summary.py $O/fpmc --kernel "6, true, true, false" --json $O/fpmc_frame.json > $O/fpmc_frame.txt 2>&1
python3 scripts/pmc_sq_summary.py $O/fpmc --kernel "1, false, true, false" --json $O/fpmc_raw.json > $O/fpmc_raw.txt 2>&1
cat $O/fpmc_frame.txt $O/fpmc_raw.txt | grep -i "valu\|wave" | head -12
find $O/fpmc -name '*counter_collection.csv' -delete
# frame launches with and without the controller-picked buffers (SQ_FRAME_TRI=0:
# buffers from the kernel arguments, a snapshot store in each frame's first launch)
for t in 1 0; do
  SQ_FRAME_TRI=$t timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ftr$t -o run --output-format csv -- python3 -u scripts/bench_rows_f.py > $O/rows_f_tri$t.log 2>&1 || { tail $O/rows_f_tri$t.log; exit 6; }
  f=$(find $O/ftr$t -name '*kernel_trace.csv' | head -1)
  python3 scripts/frame_timeline.py "$f" > $O/frame_timeline_tri$t.txt 2>&1; echo "tri=$t"; cat $O/frame_timeline_tri$t.txt
  find $O/ftr$t -name '*kernel_trace.csv' -delete
done
