#!/bin/bash
# Round 6 closing call: the whole GPU suite, smoke, the driver's command twice,
# and the driver's N = 8 launcher (torch.distributed.run, 8 ranks) rehearsed
# on one GPU with --same-device.
set -o pipefail
cd "${GRAFT_REPO_ROOT}" || exit 1
O=gpurun_out/${1:-r06_final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 \
  || { tail -40 $O/suite.log; exit 2; }
tail -1 $O/suite.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail -5 $O/bench_driver_$r.log; exit 4; }
done
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --same-device --steps 20 --warmup 5 > $O/torchrun_8.log 2>&1 || { tail -20 $O/torchrun_8.log; exit 5; }
python3 - <<PY
import json
for f in ("bench_driver_1", "bench_driver_2", "torchrun_8"):
    d = json.loads([l for l in open("$O/%s.log" % f) if l.startswith("{")][-1]); rl = d["roofline"]
    line = [f, "%.4e" % d["value"], round(d["ms_per_step"] * 1e3, 2), rl["bound"], rl.get("frac"), rl.get("launch_us_vs_rocprof_avg"),
            rl.get("profile_timing_mismatch"), d["multi_rank_check"], d["oracle_check"], d.get("oracle_check_noise")]
    c5 = d.get("c5_1024", {})
    line += ["c5 %.3e" % c5.get("value", 0), c5.get("multi_rank_check"), c5.get("oracle_check"), c5.get("oracle_check_noise")]
    if "c3_512" in d:
        line += ["c3 %.3e" % d["c3_512"]["value"], d["c3_512"]["roofline"].get("launch_us_vs_rocprof_avg"),
                 "c1 %.3e" % d["c1_qm1d"]["value"], "frames", d["frames_256"]["overhead"],
                 "slab", d["slab_1gpu"]["rccl"].get("ratio_to_single"), d["slab_1gpu"]["p2p"].get("ratio_to_single"),
                 "c1phi4", d["c1_phi4_32"].get("tauhost_equals_library")]
    print(*line)
PY
