#!/bin/bash
# Serial-order frame time vs the sweep's publication interval (SQ_GS_PUBLISH).
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for P in 8 32 128 100000; do
  echo "publish=$P"
  SQ_GS_PUBLISH=$P timeout -k 10 200 python3 "$R/scripts/bench_qm1d.py" --ordering serial --frames 3 | grep '^{' | cut -c1-110
done
