#!/bin/bash
# Round-6 profile of EXACTLY the driver's bench invocation
# (`python3 bench.py --steps 20 --warmup 5`): rocprofv3 kernel-trace stats, then
# PMC passes one counter group per run (FETCH_SIZE; WRITE_SIZE; SQ), summarised
# by scripts/driver_profile.py into driver_profile.json -- the record bench.py's
# roofline reads (profiles/r06/driver_profile.json).  Then the same command
# twice without the profiler, reading that record.
#   bash scripts/r06/driver_prof.sh OUT_TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
O=gpurun_out/${1:-r06_prof}
mkdir -p $O profiles/r06
B="bench.py --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 2; }
grep '^{' $O/trace.log > /dev/null || { tail -20 $O/trace.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 $B > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 5; }
python3 scripts/driver_profile.py --trace $O/trace --fetch $O/fetch --write $O/write --sq $O/sq --out $O/driver_profile.json > $O/summary.log 2>&1 || { tail -20 $O/summary.log; exit 6; }
cp $O/driver_profile.json profiles/r06/driver_profile.json
cp $(find $O/trace -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
# keep the per-dispatch trace out of the merge-back (tens of MB)
find $O -name '*kernel_trace.csv' -delete
find $O -name '*counter_collection.csv' -size +20M -delete
for r in 1 2; do
  timeout -k 10 300 python3 $B > $O/bench_driver_$r.log 2>&1 || { tail -20 $O/bench_driver_$r.log; exit 7; }
done
python3 - <<EOF
import json
for f in ["$O/trace.log", "$O/bench_driver_1.log", "$O/bench_driver_2.log"]:
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); r = d["roofline"]
            print(f.split("/")[-1], "%.4e" % d["value"], round(d["ms_per_step"] * 1e3, 3), "us/step", r["bound"],
                  "frac", r["frac"], r.get("stale_profile"), "alg", r.get("frac_algorithmic"), "hbm_real", r.get("frac_hbm_real"),
                  "launch_us", r.get("avg_launch_us"), "vs_rocprof", r.get("launch_us_vs_rocprof_avg"), "mismatch", r.get("profile_timing_mismatch"),
                  "busy", r.get("busy_fraction"), "MHz", r.get("clock_MHz_measured"),
                  "| checks", d.get("multi_rank_check"), d.get("oracle_check"), d.get("oracle_check_noise"),
                  "| c3", "%.4e" % d["c3_512"]["value"], d["c3_512"]["roofline"]["frac"], d["c3_512"]["roofline"].get("launch_us_vs_rocprof_avg"),
                  "| c1", d.get("c1_qm1d", {}).get("value"),
                  "| frames", d.get("frames_256", {}).get("us_per_frame"), d.get("frames_256", {}).get("overhead"),
                  "| slab", json.dumps({k: v.get("ratio_to_single") for k, v in d.get("slab_1gpu", {}).items() if isinstance(v, dict)}),
                  "| c1_phi4_32", d.get("c1_phi4_32", {}).get("tauhost_equals_library"))
EOF
