#!/bin/bash
# Round 5, call 15: per-phase stamps of the C1 grid kernel with per-block records.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c15}
mkdir -p $O
rm -f $O/stamps.txt
SQ_QM1D_STAMPS=$O/stamps.txt timeout -k 10 120 python3 scripts/bench_c1.py --frames 2 > $O/st.log 2>&1 || exit 5
python3 scripts/c1_stamps.py $O/stamps.txt
