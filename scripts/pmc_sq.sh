#!/bin/bash
# SQ instruction-mix / busy counters for the step kernel (separate --pmc passes).
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE=${1:-256}
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$R/gpurun_out/pmcsq_$i" -o run --output-format csv \
     -- python3 "$R/scripts/diag_phi4.py" steps --size $SIZE --steps 20 || echo "pass $i failed"
done
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(R + "/gpurun_out/pmcsq_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "phi4_step" in row["Kernel_Name"]:
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(agg.items()):
    v = v[len(v) // 4:]
    print(k, sum(v) / len(v))
PY
