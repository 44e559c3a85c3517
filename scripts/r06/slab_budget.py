"""Per-block time budget of the slab path from rocprofv3 kernel traces
(scripts/r06/slab_trace.py): for the last `nblk` 16-step blocks of a run, the
block span, the compute kernels' busy time on the interior stream, the gaps
on it (cross-stream waits / event records), the exchange kernel's time and
how much of it overlaps compute.  Compared with the single slab's 16 steps.

    python scripts/r06/slab_budget.py single.csv rccl.csv [p2p.csv]
"""
import csv
import sys


def kernels(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        if "moments" in n or "rocclr" in n.lower() or "copy" in n.lower() and "nccl" not in n.lower():
            continue
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r.get("Queue_Id", r.get("Stream_Id", ""))))
    ks.sort()
    return ks


def summarize(path, steps_per_block=16, nblk=8):
    ks = kernels(path)
    phi = [k for k in ks if "phi4" in k[2]]
    other = [k for k in ks if "phi4" not in k[2]]
    # the last launches of the run: take the window of the last nblk blocks by
    # counting fused-pair steps (each phi4_tb2 launch = 2 steps of some range)
    t_end = phi[-1][1]
    # window: last nblk*steps_per_block/2 "full" pair launches approximated by time
    per = {}
    for s, e, n, q in phi:
        per.setdefault(q, []).append((s, e, n))
    qa = max(per, key=lambda q: len(per[q]))        # the interior stream: most launches
    la = per[qa]
    return ks, phi, other, qa, la, t_end


def main():
    single = sys.argv[1]
    steps_per_block = 16
    ks, phi, _, qa, la, t_end = summarize(single)
    # single slab: mean launch period of the last 80 launches (2 steps each)
    tail = la[-80:]
    per_pair = (tail[-1][1] - tail[0][0]) / 1e3 / len(tail)
    busy = sum(e - s for s, e, _ in tail) / 1e3 / len(tail)
    print(f"single: {per_pair:.2f} us per pair launch ({per_pair / 2:.2f} us/step), busy {busy:.2f} us, "
          f"gap {per_pair - busy:.2f} us")
    for path in sys.argv[2:]:
        ks, phi, other, qa, la, t_end = summarize(path)
        # blocks: the exchange kernels / copies mark block starts; use the other-queue phi4 or nccl kernels
        xk = [k for k in ks if "nccl" in k[2].lower()]
        print(f"== {path}: {len(phi)} phi4 launches, {len(xk)} exchange kernels, interior queue {qa}")
        # take the last 8 exchanges' starts as block boundaries (or for p2p, gaps)
        bounds = [k[0] for k in xk][-9:] if len(xk) >= 9 else None
        if bounds is None:
            print("  no exchange kernels (P2P copies run on the copy engines): whole-window numbers only")
            w0 = la[-64][0]
            w1 = la[-1][1]
            busy = sum(e - s for s, e, _ in la[-64:]) / 1e3
            print(f"  last 64 interior launches: span {(w1 - w0) / 1e3:.1f} us, busy {busy:.1f} us")
            continue
        for b0, b1 in zip(bounds[:-1], bounds[1:]):
            inb = [(s, e, n) for s, e, n in la if b0 - 50000 <= s < b1 - 50000]
            span = (b1 - b0) / 1e3
            busy = sum(e - s for s, e, _ in inb) / 1e3
            xs = [k for k in xk if b0 <= k[0] < b1]
            xdur = sum(k[1] - k[0] for k in xs) / 1e3
            durs = " ".join(f"{(e - s) / 1e3:.1f}" for s, e, _ in inb)
            gaps = " ".join(f"{(inb[i + 1][0] - inb[i][1]) / 1e3:.1f}" for i in range(len(inb) - 1))
            print(f"  block span {span:.1f} us ({span / steps_per_block:.2f} us/step); interior busy {busy:.1f}; "
                  f"exchange kernel {xdur:.1f}\n    launches: {durs}\n    gaps:     {gaps}")


if __name__ == "__main__":
    main()
