"""Where a QM1D grid-kernel step goes (SQ_QM1D_STAMPS text: block step t0..t4,
100 MHz ticks): per phase, the median over blocks and steps 4..63 of
  phase 1 (site updates, stores)       t1 - t0
  barrier (arrive -> released)         t2 - t1
  previous scan's outcome (loads)      t3 - t2
  scan of this step                    t4 - t3
  rest (omega, swap -> next start)     t0(j+1) - t4(j)
and the spread of t1 (arrival) over blocks per step.
    python scripts/c1_stamps.py stamps.txt"""
import collections
import statistics
import sys


def main():
    rows = [list(map(int, ln.split())) for ln in open(sys.argv[1]) if ln.strip()]
    by = collections.defaultdict(dict)
    for b, j, *t in rows:
        by[j][b] = t
    ph = collections.defaultdict(list)
    spread = []
    for j in range(4, 63):
        if j not in by or j + 1 not in by:
            continue
        arr = [t[1] for t in by[j].values()]
        spread.append((max(arr) - min(arr)) * 1e-2)
        for b, t in by[j].items():
            ph["phase1"].append((t[1] - t[0]) * 1e-2)
            ph["barrier"].append((t[2] - t[1]) * 1e-2)
            ph["outcome"].append((t[3] - t[2]) * 1e-2)
            ph["scan"].append((t[4] - t[3]) * 1e-2)
            if b in by[j + 1]:
                ph["rest"].append((by[j + 1][b][0] - t[4]) * 1e-2)
                ph["step"].append((by[j + 1][b][0] - t[0]) * 1e-2)
    print(f"blocks {len(by[4])}, frames' steps 4..62")
    for k in ("phase1", "barrier", "outcome", "scan", "rest", "step"):
        v = ph[k]
        print(f"  {k:8s} median {statistics.median(v):6.2f} us  mean {statistics.fmean(v):6.2f}")
    print(f"  arrival spread over blocks: median {statistics.median(spread):.2f} us")


if __name__ == "__main__":
    main()
