#!/bin/bash
# Round 5: the whole GPU suite, smoke, and the driver's bench command twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 2; }
tail -1 $O/suite.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail -5 $O/bench_driver_$r.log; exit 4; }
done
python3 - <<PY
import json
for r in (1, 2):
    d = json.loads([l for l in open("$O/bench_driver_%d.log" % r) if l.startswith("{")][0]); rl = d["roofline"]
    print(r, "%.4e" % d["value"], round(d["ms_per_step"] * 1e3, 2), rl["bound"], rl["frac"], rl.get("stale_profile"),
          d["multi_rank_check"], d["oracle_check"], "c3 %.3e" % d["c3_512"]["value"], "c1 %.3e" % d["c1_qm1d"]["value"],
          "c5 %.3e" % d["c5_1024"]["value"], d["c5_1024"]["oracle_check"], "frames", d["frames_256"]["overhead"],
          "slab", d["slab_1gpu"]["rccl"].get("ratio_to_single"), d["slab_1gpu"]["p2p"].get("ratio_to_single"),
          "c1phi4", d["c1_phi4_32"].get("tauhost_equals_library"))
PY
