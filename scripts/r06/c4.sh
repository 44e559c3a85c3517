#!/bin/bash
# Round 6 call 4: slab schedule sweep (RCCL / P2P self-exchange) and the frame
# variants (fold / three buffers) with the interleaved frames diagnostic.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c4}
mkdir -p $O
timeout -k 10 400 python3 scripts/r06/slab_sweep.py 1000 > $O/slab_sweep.log 2>&1 || { tail -20 $O/slab_sweep.log; exit 2; }
grep '"rep": 1' $O/slab_sweep.log
for v in "SQ_FRAME_FOLD=0" "SQ_FRAME_TRI=0"; do
  env $v timeout -k 10 200 python3 scripts/r06/frames_diag.py > $O/frames_$v.log 2>&1 || { tail -20 $O/frames_$v.log; exit 3; }
  echo $v; grep alternate $O/frames_$v.log
done
