#!/bin/bash
# Fused tests, then the slab path (RCCL self-exchange / loopback) with and without two-step fusion.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_phi4.py -x -q --timeout 120 --timeout-method thread -k "fused or deep_halo or rccl or loopback or ghost or uneven" > gpurun_out/slab_tests.log 2>&1 || { tail -40 gpurun_out/slab_tests.log; exit 1; }
tail -2 gpurun_out/slab_tests.log
for f in 0 1; do for c in rccl loopback; do
  SQ_FUSE2=$f timeout -k 10 200 python bench.py --no-cpu-baseline --comm $c --steps 1000 --warmup 500 > gpurun_out/slab_${c}_f$f.log 2>&1 || { cat gpurun_out/slab_${c}_f$f.log; exit 1; }
  echo "$c fuse=$f $(grep -o '"ms_per_step": [0-9.]*\|"ghost_depth": [0-9]*' gpurun_out/slab_${c}_f$f.log | tr '\n' ' ')"
done; done
