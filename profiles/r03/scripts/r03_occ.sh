#!/bin/bash
# Blocks per CU for the fused kernels, then SQ counters of both kernels at 256^3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r03_occ
mkdir -p $O
B="bench.py --steps 2000 --warmup 200 --settle-ms 800 --no-cpu-baseline --no-c3 --no-check"
for cfg in "0 2" "1 2" "1 3" "1 4"; do
  set -- $cfg
  SQ_TB2_PIPE=$1 SQ_TB2_BLOCKS_PER_CU=$2 timeout -k 10 120 python $B > $O/b256_p$1_bpc$2.log 2>&1 || exit 2
done
for cfg in "1 2" "1 3"; do
  set -- $cfg
  SQ_TB2_PIPE=$1 SQ_TB2_BLOCKS_PER_CU=$2 timeout -k 10 120 python bench.py --size 512 --steps 200 --warmup 20 --settle-ms 800 --no-cpu-baseline --no-check > $O/b512_p$1_bpc$2.log 2>&1 || exit 3
done
for f in $O/b*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$f'.split('/')[-1], round(d['ms_per_step']*1e3,3),'us/step', '%.3e'%d['value'], r['avg_launch_us'], r['kernel'][:60])
"; done
P="bench.py --steps 300 --warmup 50 --settle-ms 300 --no-cpu-baseline --no-c3 --no-check"
for p in 0 1; do
  SQ_TB2_PIPE=$p timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq1_p$p -o run --output-format csv -- python3 $P > $O/sq1_p$p.log 2>&1 || exit 4
  SQ_TB2_PIPE=$p timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM -d $O/sq2_p$p -o run --output-format csv -- python3 $P > $O/sq2_p$p.log 2>&1 || exit 5
  SQ_TB2_PIPE=$p timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq3_p$p -o run --output-format csv -- python3 $P > $O/sq3_p$p.log 2>&1 || exit 6
done
echo done
