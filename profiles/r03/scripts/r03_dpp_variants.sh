#!/bin/bash
# Frame launches vs raw steps (scripts/diag_fr_sites.py) for DPP-hazard diagnostic builds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${OUT:-r03_dppvar}
mkdir -p $O
for v in ${VARS:-main nop nocomb lgkm}; do
  if [ $v = main ]; then unset SQ_LIB; else export SQ_LIB=stochquant_amd/lib/variants/libstochquant_$v.so; fi
  for p in 1 0; do
    SQ_TB2_PIPE=$p timeout -k 10 120 python -u scripts/diag_fr_sites.py 4 1.0 1 ${REPS:-6} > $O/${v}_p$p.log 2>&1 || exit 1
    echo "$v pipe$p: $(grep -c 'ndiff 0 ' $O/${v}_p$p.log)/${REPS:-6} clean"
  done
done
