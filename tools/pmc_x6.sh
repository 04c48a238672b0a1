#!/bin/bash
# PMC passes over the x6 GEMM microbenchmark, one shape and tile:
#   bash tools/pmc_x6.sh fc2-badd 6   -> gpurun_out/pmc_x6/<shape>_<tile>/{p1,p2,p3}
# p1: MFMA busy / wave cycles / waits, p2: clock, LDS and VALU instruction mix,
# p3: HBM fetch (gfx950: read bytes = 2 x FETCH_SIZE)
SH=${1:-fc2-badd}; T=${2:-6}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/pmc_x6/${SH}_$T && mkdir -p $O
timeout -k 10 120 tools/bin/gemm_x6_bench $SH $T > $O/plain.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA --kernel-trace -d $O/p1 -o p1 -f csv -- tools/bin/gemm_x6_bench $SH $T > $O/p1.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --kernel-trace -d $O/p2 -o p2 -f csv -- tools/bin/gemm_x6_bench $SH $T > $O/p2.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/p3 -o p3 -f csv -- tools/bin/gemm_x6_bench $SH $T > $O/p3.txt 2>&1
