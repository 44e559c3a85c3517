#!/bin/bash
# Round-end evidence on one GPU, every step under its own time limit, stopping
# at the first failure:  bash scripts/round_evidence.sh TAG
#   1. the GPU test suite                       tests.log
#   2. bench.py with the driver's arguments      bench_driver.log
#      and the 2000-step default                 bench_2000.log
#   3. rocprofv3 kernel trace + stats of bench   trace/ (kernel_stats.csv)
#   4. PMC passes, one counter group per run     fetch/ write/ sq/ (MI355X_MICROARCH.md)
#   5. the other BASELINE sizes                  bench_512.log bench_1024.log bench_rccl_self_256.log
# Outputs under gpurun_out/evidence_TAG/.
set -o pipefail
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/evidence_$TAG
mkdir -p $O
B="bench.py --steps 400 --warmup 100 --settle-ms 300 --no-cpu-baseline"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_2000.log 2>&1 || exit 3
grep -h '^{' $O/bench_driver.log $O/bench_2000.log | cut -c1-400
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 2000 --no-cpu-baseline > $O/trace.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 || exit 6
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq -o run --output-format csv -- python3 $B > $O/sq.log 2>&1 || exit 7
timeout -k 10 150 python3 bench.py --size 512 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_512.log 2>&1 || exit 8
timeout -k 10 150 python3 bench.py --size 1024 --steps 100 --warmup 10 --settle-ms 500 --no-cpu-baseline > $O/bench_1024.log 2>&1 || exit 9
timeout -k 10 150 python3 bench.py --comm rccl --steps 1600 --warmup 200 --no-cpu-baseline > $O/bench_rccl_self_256.log 2>&1 || exit 10
grep -h '^{' $O/bench_512.log $O/bench_1024.log $O/bench_rccl_self_256.log | cut -c1-300
echo done
