#!/bin/bash
# Round-4 call 9: (1) is the slab path host-bound (scripts/diag_slab_host.py);
# (2) the sustained clock at 256^3 and 512^3: rocm-smi sampled while a long
# bench runs (the 512^3 launches ran 13 % faster in the PMC pass than in the
# sustained trace).  Stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_c9}
mkdir -p $O
timeout -k 10 240 python3 -u scripts/diag_slab_host.py > $O/slab_host.log 2>&1 || { tail $O/slab_host.log; exit 1; }
cat $O/slab_host.log
timeout -k 5 20 rocm-smi --showclocks --showpower > $O/smi_idle.log 2>&1; echo "smi rc=$?"
for cfg in "256 150000" "512 20000"; do
  set -- $cfg
  ( for i in $(seq 1 60); do echo "t=$SECONDS"; timeout -k 2 5 rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|fclk|mclk|Power \(|Socket"; sleep 0.2; done ) > $O/smi_$1.log 2>&1 &
  SMI=$!
  timeout -k 10 200 python3 bench.py --size $1 --steps $2 --warmup 100 --settle-ms 1500 --no-cpu-baseline --no-c3 --no-c1 --no-check > $O/bench_$1.log 2>&1; rc=$?
  kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
  [ $rc -eq 0 ] || { tail $O/bench_$1.log; exit 2; }
  echo "size $1 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$1.log) $(grep -c sclk $O/smi_$1.log) samples"
  grep sclk $O/smi_$1.log | sort | uniq -c | sort -rn | head -8
done
