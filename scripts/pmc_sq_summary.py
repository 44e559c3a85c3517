"""Median per-launch SQ/GRBM counters of one kernel from rocprofv3 --pmc CSVs,
plus the derived issue fractions (MI355X_MICROARCH.md §rocprofv3 PMC slots:
SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; WAIT_ANY +
WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).

    python scripts/pmc_sq_summary.py DIR [DIR ...] --kernel phi4_tb2 [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="phi4_")
    ap.add_argument("--json")
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    meta = {}
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if a.kernel in r["Kernel_Name"]:
                        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
                        vals["_duration_us"].append(dur)
                        meta = {"kernel": r["Kernel_Name"], "vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                                "lds": r["LDS_Block_Size"], "grid": r["Grid_Size"], "wg": r["Workgroup_Size"]}
    med = {}
    for k, v in vals.items():
        v = v[len(v) // 5:] if len(v) >= 10 else v  # drop the cold first launches
        med[k] = statistics.median(v)
    out = {"meta": meta, "median_per_launch": med}
    d = {}
    if "SQ_WAVE_CYCLES" in med:
        wc = med["SQ_WAVE_CYCLES"]
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
            if k in med:
                d[k + "/WAVE_CYCLES"] = med[k] / wc
    if "SQ_INSTS_VALU" in med and "SQ_WAVES" in med:
        d["VALU_insts_per_wave"] = med["SQ_INSTS_VALU"] / med["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in med and "_duration_us" in med:
        d["eff_clock_GHz"] = med["GRBM_GUI_ACTIVE"] / 8 / (med["_duration_us"] * 1e3)
    if "SQ_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        d["SQ_BUSY/GRBM_GUI_ACTIVE"] = med["SQ_BUSY_CYCLES"] / med["GRBM_GUI_ACTIVE"]
    if "SQ_INSTS_VALU" in med and "_duration_us" in med and "GRBM_GUI_ACTIVE" in med:
        # VALU issue slots: 256 CUs x 4 SIMDs, one wave-instruction per SIMD per
        # 4 cycles at full rate (v_add/v_fma issue cost 4 cyc, guide ISSUE-cost row)
        cyc = med["GRBM_GUI_ACTIVE"] / 8
        d["VALU_issue_frac_at_4cyc"] = med["SQ_INSTS_VALU"] * 4 / (1024 * cyc)
    out["derived"] = d
    s = json.dumps(out, indent=1)
    print(s)
    if a.json:
        with open(a.json, "w") as fh:
            fh.write(s)


if __name__ == "__main__":
    main()
