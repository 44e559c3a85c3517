import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from stochquant_amd import Phi4Lattice
with Phi4Lattice((256, 256, 256), dtau=0.01, m2=1.0, lam=1.0, loops=20) as lat:
    lat.init_field(0.1)
    lat.step(400); lat.sync()
    for _ in range(30):
        lat.run_frame()
    lat.sync()
