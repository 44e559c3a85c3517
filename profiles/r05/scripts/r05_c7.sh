#!/bin/bash
# Round 5, call 7: per-phase stamps of the QM1D grid kernel (C1), counter and
# flag barriers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c7}
mkdir -p $O
for b in 1 3; do
  rm -f $O/stamps_bar$b.txt
  SQ_QM1D_BAR=$b SQ_QM1D_STAMPS=$O/stamps_bar$b.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/c1_bar$b.log 2>&1 || { tail -5 $O/c1_bar$b.log; exit 2; }
  echo "bar=$b"; python3 scripts/c1_stamps.py $O/stamps_bar$b.txt
done
