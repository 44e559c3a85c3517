#!/bin/bash
# Frame records' |phi'| prefilter: phi4 GPU tests, then the interleaved frame-row A/B
# against the build before (SQ_LIB variant libstochquant_allrec.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_s2_mo}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py tests/test_gpu_p2p.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
bash scripts/r03_s2_fown_ab.sh ${1:-r03_s2_mo}/ab
