#!/bin/bash
# Round 5, call 13: the QM1D defaults (sc1 flag barrier, automatic sites per
# thread): every QM1D / serial / tauhost GPU test, C1 timing, the driver's bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c13}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_qm1d.py tests/test_gpu_qm1d_serial.py tests/test_gpu_tauhost.py > $O/qm1d.log 2>&1 || { tail -30 $O/qm1d.log; exit 3; }
tail -1 $O/qm1d.log
for r in 1 2; do
  timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_$r.log 2>&1 || { tail -5 $O/c1_$r.log; exit 4; }
  echo "c1 default run=$r $(grep '^{' $O/c1_$r.log)"
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 5; }
python3 -c "
import json
d=json.loads([l for l in open('$O/bench_driver.log') if l.startswith('{')][0])
c=d['c1_qm1d']; print('headline %.4e'%d['value'], 'c1 %.4e'%c['value'], c['ms_per_frame'], c['roofline']['frac'], (c.get('cpu_baseline') or {}).get('value'))"
