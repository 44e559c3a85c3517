# Two-step fused kernel: tests, then per-step time vs output planes per block (Z) and register budget (WPE).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_phi4.py -x -q --timeout 120 --timeout-method thread -k "fused" > gpurun_out/fuse_tests.log 2>&1 || { tail -30 gpurun_out/fuse_tests.log; exit 1; }
SQ_FUSE2=0 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 --warmup 1000 > gpurun_out/fz_ref.log 2>&1 || exit 1
for w in 1 8; do for z in 11 12 16 22; do SQ_FUSE2=1 SQ_FUSE2_Z=$z SQ_FUSE2_WPE=$w timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1000 --warmup 1000 > gpurun_out/fz_${w}_$z.log 2>&1 || exit 1; done; done
