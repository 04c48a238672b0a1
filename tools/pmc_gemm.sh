#!/bin/bash
# PMC passes over the GEMM microbenchmark (one kernel shape), rocpd output under gpurun_out/pmc_gemm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_gemm
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --kernel-trace -d gpurun_out/pmc_gemm/p1 -o p1 -- tools/bin/gemm_bench ${1:-fc1} > gpurun_out/pmc_gemm/p1.txt 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES --kernel-trace -d gpurun_out/pmc_gemm/p2 -o p2 -- tools/bin/gemm_bench ${1:-fc1} > gpurun_out/pmc_gemm/p2.txt 2>&1
