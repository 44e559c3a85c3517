#!/bin/bash
# Frame-cost A/B of library builds (SQ_LIB): scripts/bench_rows_f.py's row f1
# (a 20-step frame vs 20 raw steps at 256^3), interleaved rounds.
#   bash scripts/frame_ab.sh "name:lib name:lib ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rnd in 1 2 3; do
  for spec in $1; do
    name=${spec%%:*}; lib=${spec#*:}
    echo "$name round $rnd: $(SQ_LIB=$lib timeout -k 10 100 python3 scripts/bench_rows_f.py --reps 40 2>&1 | grep f1)"
  done
done
