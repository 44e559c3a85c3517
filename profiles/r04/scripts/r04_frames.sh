#!/bin/bash
# Round-4: device frames with the end folded into the next frame's first
# launch -- the frame tests (bitwise vs host-decided frames), then the
# 20-step 256^3 frame rows, fold on vs off interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_frames}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "frame or stab or guard or snapshot or checkpoint" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 2; }
tail -1 $O/frame_tests.log
for r in 1 2 3; do for f in 1 0; do
  SQ_FRAME_FOLD=$f timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f_fold${f}_$r.log 2>&1 || { tail $O/rows_f_fold${f}_$r.log; exit 3; }
  echo "fold=$f run=$r $(grep -h 'f1\|frames' $O/rows_f_fold${f}_$r.log | head -3 | tr '\n' ' ')"
done; done
