"""Where a batched 20-step frame's time goes, from a rocprofv3 kernel trace of
scripts/bench_rows_f.py (raw steps, then sq_run_frame x reps, then three
sq_run_frames(100) batches, then host-decided frames).  Takes the middle 100
frames of the batches (frame launches 1200..2200 after the 10 x reps of the
per-frame row) and prints, per frame: the span, the summed durations of the
frame launches, of every other kernel in the window, and the idle time.

    python scripts/frame_timeline.py run_kernel_trace.csv [--reps 20] [--per-frame 10]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--per-frame", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows),
                key=lambda t: t[0])
    # frame launches: the fused kernel's frame instances (FR template argument true)
    def is_frame(name):
        if "phi4_tb2" not in name:
            return False
        args = name.split("<", 1)[1].split(">")[0].split(", ")
        return len(args) >= 4 and args[3] == "true"

    fr = [k for k in ks if is_frame(k[2])]
    lo = a.reps * a.per_frame + 1000
    sel = fr[lo:lo + 100 * a.per_frame]
    t0, t1 = sel[0][0], sel[-1][1]
    win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
    busy, by = 0, collections.Counter()
    cnt = collections.Counter()
    last_end = t0
    for s, e, n in win:
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
        short = n.replace("void sq::(anonymous namespace)::", "")[:80]
        by[short] += e - s
        cnt[short] += 1
    nf = len(sel) / a.per_frame
    print(f"frames {nf:.0f}  span/frame {(t1 - t0) / 1e3 / nf:.1f} us  busy/frame {busy / 1e3 / nf:.1f} us  "
          f"idle/frame {(t1 - t0 - busy) / 1e3 / nf:.1f} us")
    for n, d in by.most_common():
        print(f"  {d / 1e3 / nf:8.2f} us/frame  {cnt[n] / nf:5.2f} launches/frame  avg {d / cnt[n] / 1e3:7.2f} us  {n}")
    # by the launch's index inside its frame (index 0 folds the previous frame's end)
    # and the gap before it (the previous kernel's end to its start)
    idx_d, idx_g = collections.defaultdict(list), collections.defaultdict(list)
    prev_end = None
    for j, (s, e, n) in enumerate(sel):
        idx_d[j % a.per_frame].append((e - s) / 1e3)
        if prev_end is not None:
            idx_g[j % a.per_frame].append((s - prev_end) / 1e3)
        prev_end = e
    print("  launch index in frame: avg duration / avg gap before it (us)")
    for i in sorted(idx_d):
        g = idx_g.get(i) or [0.0]
        print(f"    {i:2d}  {sum(idx_d[i]) / len(idx_d[i]):7.2f}  {sum(g) / len(g):6.2f}")
    raw = [k for k in ks if "phi4_tb2" in k[2] and not is_frame(k[2]) and "<true," in k[2]]
    if raw:
        d = sorted((e - s) / 1e3 for s, e, _ in raw)
        print(f"  raw instance: {len(raw)} launches, median {d[len(d) // 2]:.2f} us, mean {sum(d) / len(d):.2f} us")


if __name__ == "__main__":
    main()
