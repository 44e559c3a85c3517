#!/bin/bash
# Round-4 call 10: the measured shader clock (block stamps with s_memtime) --
# its test, then the driver's invocation twice; a kernel trace of the frame
# rows (scripts/frame_timeline.py: where a batched frame's time goes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c10}
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_phi4.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "block_stamps" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail $O/bench_driver_$r.log; exit 2; }
  python3 - $O/bench_driver_$r.log <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][0])
r, c = d["roofline"], d["c3_512"]["roofline"]
print(d["value"], d["ms_per_step"], r["frac"], r.get("clock_MHz_measured"), r.get("frac_at_measured_clock"), r.get("busy_fraction"),
      "| c3", d["c3_512"]["value"], c["frac"], c.get("clock_MHz_measured"), c.get("frac_at_measured_clock"), c.get("busy_fraction"))
EOF
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ftr -o run --output-format csv -- python3 -u scripts/bench_rows_f.py > $O/rows_f_trace.log 2>&1 || { tail $O/rows_f_trace.log; exit 3; }
f=$(find $O/ftr -name '*kernel_trace.csv' | head -1)
python3 scripts/frame_timeline.py "$f" > $O/frame_timeline.txt 2>&1; cat $O/frame_timeline.txt
cp $(find $O/ftr -name '*kernel_stats.csv' | head -1) $O/rows_f_kernel_stats.csv
find $O/ftr -name '*kernel_trace.csv' -delete
