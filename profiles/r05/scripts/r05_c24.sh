#!/bin/bash
# Round 5, call 24: how long the split-barrier kernel's slack work takes
# (SQ_QM1D_PSLEEP=2 moves the third stamp from after the wait to the end of the
# slack work), against the default stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c24}
mkdir -p $O
for ps in 2 1; do
  rm -f $O/stamps_s$ps.txt
  SQ_QM1D_PSLEEP=$ps SQ_QM1D_STAMPS=$O/stamps_s$ps.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st_s$ps.log 2>&1 || exit 5
  echo "stamps psleep=$ps"; python3 scripts/c1_stamps.py $O/stamps_s$ps.txt
done
