#!/bin/bash
# Round 6 call 30: RCCL's kernel time per self-exchange, faces whole (k = 1)
# and split in 2 / 4 / 8 (SQ_RCCL_SPLIT), from kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c30}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 4 8; do
  SQ_RCCL_SPLIT=$k timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_s$k -o run -- python3 scripts/r06/slab_trace.py rccl 320 > $O/tr_s$k.log 2>&1 || { tail -20 $O/tr_s$k.log; exit 3; }
  python3 - $O/tr_s$k/run_kernel_trace.csv $k <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
r = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000 for x in rows if "rccl" in x["Kernel_Name"].lower() or "nccl" in x["Kernel_Name"].lower()]
t = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000 for x in rows if "tb2_kernel" in x["Kernel_Name"]]
r = r[len(r) // 3:]
print("split", sys.argv[2], "rccl kernels", len(r), "mean us %.2f" % (sum(r) / max(1, len(r))), "median %.2f" % sorted(r)[len(r) // 2] if r else "", "tb2 mean %.2f" % (sum(t) / max(1, len(t))))
PY
done
