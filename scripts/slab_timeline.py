"""Per-block breakdown of a slab-path kernel trace (scripts/trace_slab_r02.sh):
the last few 16-step blocks of the timed region, every kernel with its start
offset, duration and the gap before it."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70], r.get("Queue_Id", ""))
             for r in rows if "copy_kernel" not in r["Kernel_Name"] and "moments" not in r["Kernel_Name"]
             and "rocclr" not in r["Kernel_Name"]), key=lambda t: t[0])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
sel = ks[-n:]
t0 = sel[0][0]
prev_end = {}
for s, e, name, q in sel:
    gap = (s - prev_end[q]) / 1e3 if q in prev_end else 0.0
    prev_end[q] = e
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  q{q:>3}  {name.replace('void sq::(anonymous namespace)::', '')}")
tot = (sel[-1][1] - sel[0][0]) / 1e3
print(f"span {tot:.1f} us over {n} kernels")
