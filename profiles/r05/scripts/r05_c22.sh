#!/bin/bash
# Round 5, call 22: the split-barrier C1 kernel, polling wave (qm1d_frame_gridp: step j+1's block-local work
# between arriving and waiting): every QM1D / serial / tauhost GPU test, C1 timing, stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c22}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_qm1d.py tests/test_gpu_qm1d_serial.py tests/test_gpu_tauhost.py > $O/qm1d.log 2>&1 || { tail -30 $O/qm1d.log; exit 3; }
tail -1 $O/qm1d.log
for r in 1 2; do
  timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_$r.log 2>&1 || { tail -5 $O/c1_$r.log; exit 4; }
  echo "c1 default run=$r $(grep '^{' $O/c1_$r.log)"
done
for r in 1 2; do
  SQ_QM1D_PIPE=0 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_plain_$r.log 2>&1 || { tail -5 $O/c1_plain_$r.log; exit 5; }
  echo "c1 plain run=$r $(grep '^{' $O/c1_plain_$r.log)"
done
rm -f $O/stamps.txt
SQ_QM1D_STAMPS=$O/stamps.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st.log 2>&1 || exit 6
python3 scripts/c1_stamps.py $O/stamps.txt
