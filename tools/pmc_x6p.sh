#!/bin/bash
# PMC passes over one x6p GEMM shape: bash tools/pmc_x6p.sh M N K EPI -> gpurun_out/pmc_x6p/<M>_<N>_<K>_<EPI>
M=$1; N=$2; K=$3; E=${4:-0}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/pmc_x6p/${M}_${N}_${K}_$E && mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --kernel-trace -d $O/p1 -o p1 -f csv -- tools/bin/gemm_x6_bench x6p $M $N $K $E > $O/p1.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS --kernel-trace -d $O/p2 -o p2 -f csv -- tools/bin/gemm_x6_bench x6p $M $N $K $E > $O/p2.txt 2>&1
