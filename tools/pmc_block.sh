#!/bin/bash
# PMC passes over the block's memory-bound kernels (FFT rows, transposes) in bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_blk
RX='fft_|transpose'
timeout -k 10 200 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/pmc_blk/p1 -o p1 -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/pmc_blk/p1.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex "$RX" --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR MeanOccupancyPerActiveCU TA_BUSY --kernel-trace -d gpurun_out/pmc_blk/p2 -o p2 -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/pmc_blk/p2.txt 2>&1
