#!/bin/bash
# Round 6 call 11: three-buffer frames that start on the host's guess of their
# buffers (SQ_FRAME_SPEC) -- the frame / stability / rollback GPU tests, then
# the frames diagnostic with the guess on and off, twice, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c11}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py \
  -k "frame or stab or rollback or guard or checkpoint or snapshot" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    SQ_FRAME_SPEC=$v timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_spec${v}_$r.log 2>&1 || { tail -20 $O/frames_spec${v}_$r.log; exit 3; }
    echo "spec=$v run $r: $(grep alternate $O/frames_spec${v}_$r.log | python3 -c 'import sys,json; print([round(json.loads(l)["overhead"],4) for l in sys.stdin])')"
  done
done
