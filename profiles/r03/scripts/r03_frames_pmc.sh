#!/bin/bash
# SQ counters of the frame vs raw fused-kernel instances at 256^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_fpmc}
mkdir -p $O
P="python3 scripts/frames_only.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq1 -o run --output-format csv -- $P > $O/sq1.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM -d $O/sq2 -o run --output-format csv -- $P > $O/sq2.log 2>&1 || exit 5
for k in "6, true, true" "1, false, true"; do
  python3 scripts/pmc_sq_summary.py $O/sq1 $O/sq2 --kernel "phi4_tb2_kernel<true, false, $k>" > "$O/sum_${k//[, ]/_}.json" || exit 6
done
ls $O
