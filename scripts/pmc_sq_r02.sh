set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 gpurun_out/pmc_sq3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_sq1 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 200 --no-cpu-baseline > gpurun_out/pmc_sq1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA -d gpurun_out/pmc_sq2 -o run --output-format csv -- python3 bench.py --steps 200 --warmup 200 --no-cpu-baseline > gpurun_out/pmc_sq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_sq3 -o run --output-format csv -- python3 bench.py --size 512 --steps 40 --warmup 40 --no-cpu-baseline > gpurun_out/pmc_sq3.log 2>&1
