#!/bin/bash
# Round-2 measurements beyond the headline: the bench line at 512^3 (C3) and
# 1024^3 (C5's lattice on one GPU), the fused-vs-per-step sweep on C5's
# per-GPU slab, the RCCL slab path, and a rocprofv3 kernel trace + PMC
# traffic of the 512^3 bench command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/sizes_r02
mkdir -p $O
timeout -k 10 150 python3 bench.py --size 512 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_512.log 2>&1 || exit 2
timeout -k 10 200 python3 bench.py --size 1024 --steps 20 --warmup 4 --settle-ms 500 --no-cpu-baseline > $O/bench_1024.log 2>&1 || exit 3
timeout -k 10 200 python3 scripts/sweep_tb2.py --shape 1024x1024x128 --variants "fuse0;fuse1,wpe6,bpc2;fuse1,wpe1,bpc2" > $O/sweep_1024x1024x128.log 2>&1 || exit 4
timeout -k 10 120 python3 bench.py --comm rccl --steps 1600 --warmup 200 --no-cpu-baseline > $O/bench_rccl_256.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/trace512 -o run --output-format csv -- python3 bench.py --size 512 --steps 200 --warmup 20 --no-cpu-baseline > $O/trace512.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch512 -o run --output-format csv -- python3 bench.py --size 512 --steps 40 --warmup 10 --settle-ms 200 --no-cpu-baseline > $O/fetch512.log 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write512 -o run --output-format csv -- python3 bench.py --size 512 --steps 40 --warmup 10 --settle-ms 200 --no-cpu-baseline > $O/write512.log 2>&1 || exit 8
echo done
