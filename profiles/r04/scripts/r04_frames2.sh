#!/bin/bash
# Round-4: three-buffer device frames (the start buffer is the rollback: no
# snapshot store, no copy back) -- the frame tests bitwise against host-decided
# frames, then the 20-step 256^3 frame rows, SQ_FRAME_TRI on/off interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r04_frames2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "frame or stab or guard or snapshot or checkpoint" > $O/frame_tests.log 2>&1 || { tail -30 $O/frame_tests.log; exit 2; }
tail -1 $O/frame_tests.log
SQ_FRAME_FOLD=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "run_frames" > $O/frame_tests_nofold.log 2>&1 || { tail -30 $O/frame_tests_nofold.log; exit 2; }
tail -1 $O/frame_tests_nofold.log
for r in 1 2 3; do for t in 1 0; do
  SQ_FRAME_TRI=$t timeout -k 10 200 python -u scripts/bench_rows_f.py > $O/rows_f_tri${t}_$r.log 2>&1 || { tail $O/rows_f_tri${t}_$r.log; exit 3; }
  echo "tri=$t run=$r $(grep -h 'f1' $O/rows_f_tri${t}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["raw_steps_us"], d["batch_frame_us"], d["frame_us"])')"
done; done
