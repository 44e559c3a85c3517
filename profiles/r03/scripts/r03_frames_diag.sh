#!/bin/bash
# Frames == raw steps, repeated, for both fused kernels (one-accumulator frame records).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r03_frames}
mkdir -p $O
SQ_TB2_PIPE=1 timeout -k 10 200 python -u scripts/diag_frames_pipe.py 3 > $O/pipe1.log 2>&1 || { tail -20 $O/pipe1.log; exit 1; }
SQ_TB2_PIPE=0 timeout -k 10 200 python -u scripts/diag_frames_pipe.py 3 > $O/pipe0.log 2>&1 || { tail -20 $O/pipe0.log; exit 2; }
grep -h "FAILED" $O/pipe1.log $O/pipe0.log
