#!/bin/bash
# Round 6 call 12: the driver's command twice on this build (sub-records with
# rotating order).
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_c12}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail -5 $O/bench_driver_$r.log; exit 4; }
done
python3 - <<PY
import json
for f in ("bench_driver_1", "bench_driver_2"):
    d = json.loads([l for l in open("$O/%s.log" % f) if l.startswith("{")][-1]); rl = d["roofline"]
    print(f, "%.4e" % d["value"], round(d["ms_per_step"] * 1e3, 2), rl.get("frac"), rl.get("launch_us_vs_rocprof_avg"),
          d["multi_rank_check"], d["oracle_check"], d.get("oracle_check_noise"), "frames", d["frames_256"]["overhead"],
          "slab", d["slab_1gpu"]["rccl"].get("ratio_to_single"), d["slab_1gpu"]["p2p"].get("ratio_to_single"))
PY
