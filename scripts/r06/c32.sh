#!/bin/bash
# Round 6 call 32: RCCL user-buffer registration of the field buffers
# (SQ_RCCL_REGISTER=1) for the in-order self-exchange: bitwise check, kernel
# time from a trace, and the interleaved A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c32}
mkdir -p $O
SQ_RCCL_REGISTER=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_phi4.py -k "rccl or exchange_on_interior" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
export TMPDIR=/tmp
SQ_RCCL_REGISTER=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_reg -o run -- python3 scripts/r06/slab_trace.py rccl 320 > $O/tr_reg.log 2>&1 || { tail -20 $O/tr_reg.log; exit 3; }
python3 - $O/tr_reg/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
r = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000 for x in rows if "rccl" in x["Kernel_Name"].lower() or "nccl" in x["Kernel_Name"].lower()]
r = r[len(r) // 3:]
print("registered: rccl kernels", len(r), "mean us %.2f" % (sum(r) / max(1, len(r))))
PY
timeout -k 10 500 python3 -u scripts/r06/slab_ab.py 1000 9 rccl:rccl rccl_reg:rccl:SQ_RCCL_REGISTER=1 > $O/slab_ab.log 2>&1 || { tail -30 $O/slab_ab.log; exit 4; }
grep '^{' $O/slab_ab.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); [print(k, v["ratio"], v["median_us"]) for k,v in d["contexts"].items()]'
