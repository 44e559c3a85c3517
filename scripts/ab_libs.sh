#!/bin/bash
# Interleaved A/B of library builds (SQ_LIB) on the fused kernel: per round and
# build, one process timing --steps steps at each shape (scripts/sweep_tb2.py).
#   bash scripts/ab_libs.sh "base:stochquant_amd/lib/libstochquant.so var:stochquant_amd/lib/variants/x.so"
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab_libs
mkdir -p $O
for rnd in 1 2 3; do
  for spec in $1; do
    name=${spec%%:*}; lib=${spec#*:}
    for shape in ${SHAPES:-256x256x256 512x512x512}; do
      SQ_LIB=$lib timeout -k 10 100 python3 scripts/sweep_tb2.py --shape $shape --steps ${STEPS:-1000} --rounds 2 \
        --variants "fuse1,wpe6,bpc2" > $O/${name}_${shape}_$rnd.log 2>&1 || exit 3
      echo "$name $shape round $rnd: $(grep 'us ' $O/${name}_${shape}_$rnd.log | tail -1)"
    done
  done
done
