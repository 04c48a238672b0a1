#!/bin/bash
# PMC passes over the block's row FFT kernels (bench.py, 2 steps): bash tools/pmc_fft.sh -> gpurun_out/pmc_fft
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/pmc_fft && mkdir -p $O
R="--kernel-include-regex fft_"
timeout -s KILL 120 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace -d $O/p1 -o p1 -f csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $O/p1.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 $R --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS --kernel-trace -d $O/p2 -o p2 -f csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $O/p2.txt 2>&1
