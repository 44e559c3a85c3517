#!/bin/bash
# Round 5, first GPU call: the new parity / boundary tests, the whole GPU
# suite, smoke, and the driver's bench invocation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c1}
mkdir -p $O
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_phi4.py::test_launch_info_names_each_instance \
  tests/test_gpu_phi4.py::test_oracle_protocol_matches_oracle tests/test_gpu_phi4.py::test_oracle_check_full_size_256 \
  tests/test_gpu_phi4.py::test_c2_hot_instance_vs_oracle tests/test_gpu_tauhost.py::test_configs0_phi4_32_through_tauhost \
  > $O/new_tests.log 2>&1 || exit 2
timeout -k 10 90 $T tests/test_gpu_qm1d.py::test_grid_barrier_timeout_returns_error > $O/barrier.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 || exit 4
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 6
