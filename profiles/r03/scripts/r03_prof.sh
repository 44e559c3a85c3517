#!/bin/bash
# Round-3 profile set of the bench commands (256^3 and 512^3): rocprofv3
# kernel-trace stats, then PMC passes one counter group per run (FETCH_SIZE;
# WRITE_SIZE; two SQ groups; GRBM), then the traffic / VALU summaries that
# bench.py reads (profiles/pmc_traffic_<L>.json).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_prof}
mkdir -p $O
for L in 256 512; do
  if [ $L = 256 ]; then S="--steps 200 --warmup 20"; else S="--steps 40 --warmup 10"; fi
  B="bench.py --size $L $S --settle-ms 300 --no-cpu-baseline --no-c3 --no-check"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats_$L -o run --output-format csv -- python3 $B > $O/stats_$L.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$L -o run --output-format csv -- python3 $B > $O/fetch_$L.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_$L -o run --output-format csv -- python3 $B > $O/write_$L.log 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq1_$L -o run --output-format csv -- python3 $B > $O/sq1_$L.log 2>&1 || exit 5
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM -d $O/sq2_$L -o run --output-format csv -- python3 $B > $O/sq2_$L.log 2>&1 || exit 6
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/grbm_$L -o run --output-format csv -- python3 $B > $O/grbm_$L.log 2>&1 || exit 7
  python3 scripts/pmc_sq_summary.py $O/sq1_$L $O/sq2_$L $O/grbm_$L --kernel phi4_tb2 --json $O/pmc_sq_$L.json > /dev/null || exit 8
  python3 scripts/pmc_traffic.py $O/fetch_$L $O/write_$L --size $L --kernel phi4_tb2 --sq $O/pmc_sq_$L.json --out $O/pmc_traffic_$L.json || exit 9
done
ls $O
