"""256^3 raw 20-step blocks and 20-step frames back to back (sq_run_frames), for
rocprofv3 --pmc passes that compare the frame and raw kernel instances."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stochquant_amd import Phi4Lattice
    with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, loops=20) as lat:
        lat.init_field(0.1)
        lat.step(400)
        lat.sync()
        for _ in range(5):
            lat.step(20)
        lat.run_frames(5)
        lat.sync()


if __name__ == "__main__":
    main()
