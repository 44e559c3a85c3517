"""Turn two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE; separate passes,
MI355X_MICROARCH.md §rocprofv3 PMC slots) into HBM bytes per launch of the
phi^4 step kernel (one step per launch) or two-step fused kernel (two), and
write profiles/pmc_traffic.json for bench.py.  algorithmic bytes = 8 B per
site update x the updates of one launch; hbm_min = one read
and one write of the field, the least any launch can move.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts the
L2's memory-side read requests at 64 B but wide streaming reads issue 128-B
requests, so it reports exactly half the bytes: multiply by 2.  WRITE_SIZE
(KiB) is exact for 16-B-per-lane streaming stores.  Infinity-Cache hits are
counted, so at 256^3 (working set < 256 MiB) this is L2-miss traffic, not
strictly DRAM traffic.

    python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR --size 256 [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics

N_SIMD = 1024        # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4      # peak engine clock (MI355X_MICROARCH.md)


def counter_values(d, counter, kernel_substr="phi4_"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    kname = None
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
                    kname = row["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_substr} in {files}")
    return vals, kname


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--kernel", default="phi4_tb2", help="kernel-name substring (phi4_tb2 or phi4_step)")
    ap.add_argument("--sq", help="a pmc_sq_summary.py --json output of the same command: its issue "
                                 "figures are recorded beside the traffic")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fv, kname = counter_values(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wv, _ = counter_values(a.write_dir, "WRITE_SIZE", a.kernel)
    # drop the first launches (cold caches) when there are enough samples
    fv_s = fv[len(fv) // 5:] if len(fv) >= 10 else fv
    wv_s = wv[len(wv) // 5:] if len(wv) >= 10 else wv
    fetch_kib = statistics.median(fv_s)
    write_kib = statistics.median(wv_s)
    read_bytes = 2.0 * fetch_kib * 1024
    write_bytes = write_kib * 1024
    # two-step fused launches (phi4_tb2_kernel) do two site updates per site
    spl = 2 if "tb2" in kname else 1
    alg = 8 * a.size ** 3 * spl
    out = {
        "size": a.size,
        "nranks": a.nranks,
        "kernel": kname,
        "launches_fetch": len(fv), "launches_write": len(wv),
        "FETCH_SIZE_KiB_median": fetch_kib,
        "WRITE_SIZE_KiB_median": write_kib,
        "read_bytes_per_launch": read_bytes,
        "write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "steps_per_launch": spl,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / alg,
        "hbm_min_bytes_per_launch": 8 * a.size ** 3,
        "traffic_over_hbm_min": (read_bytes + write_bytes) / (8 * a.size ** 3),
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streaming reads), KiB x1024",
    }
    if a.sq:
        with open(a.sq) as fh:
            sq = json.load(fh)
        med, der = sq["median_per_launch"], sq["derived"]
        out["sq_source"] = a.sq
        out["valu_insts_per_wave"] = der.get("VALU_insts_per_wave")
        dur = med.get("_duration_us")
        if dur and "SQ_ACTIVE_INST_VALU" in med:
            # per-SIMD VALU utilisation over the kernel span: the VALU issue
            # cycles of all waves (SQ_ACTIVE_INST_VALU counts quad-cycles) over
            # 1024 SIMDs x the launch's cycles at the 2.4 GHz peak engine clock
            # (a lower bound if the clock ran below peak); issue-cost form: one
            # wave64 VALU instruction = 4 cycles (SQ_INSTS_VALU x 4)
            cyc = CLOCK_GHZ * 1e3 * dur
            out["pmc_kernel_us"] = round(dur, 3)
            out["valu_util_simd"] = round(4.0 * med["SQ_ACTIVE_INST_VALU"] / (N_SIMD * cyc), 3)
            out["valu_issue_util_simd"] = round(4.0 * med["SQ_INSTS_VALU"] / (N_SIMD * cyc), 3)
            if "SQ_WAVE_CYCLES" in med:
                out["avg_resident_waves_per_simd"] = round(4.0 * med["SQ_WAVE_CYCLES"] / (N_SIMD * cyc), 2)
            out["valu_util_method"] = (f"SQ_ACTIVE_INST_VALU x 4 / ({N_SIMD} SIMDs x {CLOCK_GHZ} GHz x "
                                       f"kernel duration of the PMC run)")
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
