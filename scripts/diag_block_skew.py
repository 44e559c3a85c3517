"""Is the fused launch's block-end spread systematic (the same blocks slow in
every launch) or random?  Per-block durations of R stamped 256^3 launches
(sq_phi4_block_stamps): the correlation of durations between launches, the
mean duration by XCD (block id mod 8), and start / end spreads.
    python scripts/diag_block_skew.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    from stochquant_amd import Phi4Lattice
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, seed=0x5EED) as lat:
        lat.init_field(0.1)
        lat.step(2000)
        lat.sync()
        D, S, E = [], [], []
        for _ in range(R):
            lat.step(300)
            st, en = lat.block_stamps()
            t0 = st.min()
            S.append((st - t0) * 1e-2)
            E.append((en - t0) * 1e-2)
            D.append((en - st) * 1e-2)
        D, S, E = np.array(D), np.array(S), np.array(E)
        nb = D.shape[1]
        print(f"blocks {nb}, launches {R}")
        print(f"span mean {E.max(1).mean():.2f} us; start max mean {S.max(1).mean():.2f}; "
              f"duration mean {D.mean():.2f} min {D.min(1).mean():.2f} max {D.max(1).mean():.2f}")
        c = np.corrcoef(D)
        print(f"corr of block durations between launches: mean off-diagonal {c[~np.eye(R, dtype=bool)].mean():.3f}")
        c2 = np.corrcoef(S)
        print(f"corr of block starts between launches: {c2[~np.eye(R, dtype=bool)].mean():.3f}")
        m = D.mean(0)
        print("mean duration by b % 8:", " ".join(f"{m[np.arange(nb) % 8 == x].mean():.2f}" for x in range(8)))
        print("block-mean duration p10/p50/p90:", np.percentile(m, [10, 50, 90]).round(2),
              " per-launch residual std:", (D - m).std().round(3))
        b = np.arange(nb)
        lb = (b & 7) * (nb >> 3) + (b >> 3)
        yb, zk = lb % 32, lb // 32
        for name, key, n in (("yb (y-band)", yb, 32), ("zk (z-chunk)", zk, 16), ("(b>>3)%32 (slot in XCD)", (b >> 3) % 32, 32),
                             ("(b>>3)//32 (1st/2nd round in XCD)", (b >> 3) // 32, 2)):
            g = np.array([m[key == v].mean() for v in range(n)])
            print(f"by {name}: spread of group means {g.max() - g.min():.2f} us;", " ".join(f"{x:.1f}" for x in g))
        # blocks sorted by start: duration of the earliest / latest quarter
        order = np.argsort(S.mean(0))
        q = nb // 4
        print("duration by start quartile:", " ".join(f"{m[order[i*q:(i+1)*q]].mean():.2f}" for i in range(4)))
        # if each block ran at its own mean speed with starts as measured
        busy = (D.sum(1) / (nb * E.max(1))).mean()
        print(f"busy fraction {busy:.3f}; span if every block took the mean duration {D.mean() + S.max(1).mean():.2f}")
        wait = (E.max(1)[:, None] - E).mean()
        print(f"mean idle tail per block {wait:.2f} us; end spread explained by start {np.corrcoef(S.ravel(), E.ravel())[0,1]:.3f}")


if __name__ == "__main__":
    main()
