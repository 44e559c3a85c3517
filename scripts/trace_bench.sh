#!/bin/bash
# Per-dispatch kernel trace of a short bench run (duration distribution of the step kernel).
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace_bench" -o run --output-format csv \
   -- python3 "$R/bench.py" --no-cpu-baseline "$@"
f=$(find "$R/gpurun_out/trace_bench" -name "*kernel_trace.csv" | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "phi4_step" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
g = [int(rows[i+1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]) for i in range(len(rows)-1)]
import statistics as st
print("n", len(d), "dur mean", st.mean(d), "median", st.median(d), "min", min(d), "max", max(d))
print("gap mean", st.mean(g), "median", st.median(g), "min", min(g), "max", max(g))
for k in range(0, len(d), 200):
    print(k, round(st.mean(d[k:k+200])), round(st.mean(g[k:k+199])) if g[k:k+199] else None)
PY
