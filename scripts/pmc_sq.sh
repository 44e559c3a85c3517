#!/bin/bash
# SQ instruction-mix / busy counters for the step kernel (separate --pmc passes).
#   scripts/pmc_sq.sh SIZE [TAG]   (KSUB: kernel-name substring, default phi4_)
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE=${1:-256}; TAG=${2:-x}
KSUB=${KSUB:-phi4_}
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d "$R/gpurun_out/pmcsq_${TAG}_$i" -o run --output-format csv \
     -- python3 "$R/scripts/diag_phi4.py" steps --size $SIZE --steps 20 || echo "pass $i failed"
done
python3 - "$R" "$TAG" "$KSUB" <<'PY'
import csv, glob, sys, collections
R, TAG, KSUB = sys.argv[1:4]
agg = collections.defaultdict(list)
for f in glob.glob(R + f"/gpurun_out/pmcsq_{TAG}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if KSUB in row["Kernel_Name"]:
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, v in sorted(agg.items()):
    v = v[len(v) // 4:]
    print(k, sum(v) / len(v))
PY
