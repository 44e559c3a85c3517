#!/bin/bash
# Two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over the step
# kernel at a given size, then the traffic summary.   scripts/pmc_run.sh SIZE TAG
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SIZE=${1:-256}; TAG=${2:-r01}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$R/gpurun_out/pmc_${SIZE}_$c" -o run --output-format csv \
     -- python3 "$R/scripts/diag_phi4.py" steps --size $SIZE --steps ${STEPS:-30}
done
python3 "$R/scripts/pmc_traffic.py" "$R/gpurun_out/pmc_${SIZE}_FETCH_SIZE" "$R/gpurun_out/pmc_${SIZE}_WRITE_SIZE" \
   --size $SIZE --out "$R/gpurun_out/pmc_traffic_${SIZE}_${TAG}.json"
cat "$R/gpurun_out/pmc_traffic_${SIZE}_${TAG}.json"
