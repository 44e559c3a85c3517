#!/bin/bash
# QM1D: GPU tests on the new build, then an interleaved A/B of Jacobi frame
# times against the round-3 base (SQ_LIB variant).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_qab}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_qm1d.py tests/test_gpu_qm1d_serial.py tests/test_gpu_tauhost.py tests/test_gpu_selftest.py > $O/qm1d_tests.log 2>&1 || { tail -30 $O/qm1d_tests.log; exit 2; }
tail -1 $O/qm1d_tests.log
for r in 1 2; do
  for v in base new; do
    lib=stochquant_amd/lib/libstochquant.so; [ $v = base ] && lib=stochquant_amd/lib/variants/libstochquant_qbase.so
    SQ_LIB=$lib timeout -k 10 200 python -u scripts/bench_qm1d.py --ordering jacobi --no-cpu --frames 10 > $O/j_${v}_$r.log 2>&1 || { tail $O/j_${v}_$r.log; exit 3; }
    echo "$v $r: $(python3 -c "
import json,sys
print(' '.join('N%d %.3f'%(d['N'],d['gpu_ms_per_frame']) for d in map(json.loads,[l for l in open('$O/j_${v}_$r.log') if l.startswith('{')])))")"
  done
done
timeout -k 10 200 python -u scripts/bench_qm1d.py --ordering serial --no-cpu --frames 10 > $O/serial_new.log 2>&1 || exit 4
cat $O/serial_new.log
