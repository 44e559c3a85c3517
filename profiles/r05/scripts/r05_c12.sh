#!/bin/bash
# Round 5, call 12: C1 with the sc1 flag barrier at 1 / 2 sites per thread.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c12}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_qm1d.py -k "c1_frames" > $O/qm1d_k1.log 2>&1 || { tail -30 $O/qm1d_k1.log; exit 3; }
tail -1 $O/qm1d_k1.log
for r in 1 2 3; do for cfg in "4 1" "4 2" "1 8"; do
  set -- $cfg
  SQ_QM1D_BAR=$1 SQ_QM1D_GK=$2 timeout -k 10 120 python3 scripts/bench_c1.py --frames 16 > $O/c1_bar$1_k$2_$r.log 2>&1 || { tail -5 $O/c1_bar$1_k$2_$r.log; exit 4; }
  echo "bar=$1 K=$2 run=$r $(grep '^{' $O/c1_bar$1_k$2_$r.log)"
done; done
rm -f $O/stamps_bar4_k1.txt
SQ_QM1D_BAR=4 SQ_QM1D_GK=1 SQ_QM1D_STAMPS=$O/stamps_bar4_k1.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st.log 2>&1 || exit 5
python3 scripts/c1_stamps.py $O/stamps_bar4_k1.txt
