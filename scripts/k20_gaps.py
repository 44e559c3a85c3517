"""Gaps inside the K = 20 regions of scripts/diag_k20_trace.py's kernel trace:
python3 scripts/k20_gaps.py DIR"""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "phi4" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
# regions: runs of launches separated by > 50 us of idle
regs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if b[0] - a[1] > 50_000:
        regs.append(cur)
        cur = []
    cur.append(b)
regs.append(cur)
for reg in regs:
    if len(reg) > 20:
        continue
    durs = [(e - s) / 1e3 for s, e, _ in reg]
    gaps = [(reg[i + 1][0] - reg[i][1]) / 1e3 for i in range(len(reg) - 1)]
    print(f"{len(reg)} launches: span {(reg[-1][1] - reg[0][0]) / 1e3:.1f} us; durations "
          + " ".join(f"{d:.1f}" for d in durs) + "; gaps " + " ".join(f"{g:.1f}" for g in gaps))
    print("   kernels:", sorted(set(k for _, _, k in reg)))
