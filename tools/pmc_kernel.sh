#!/bin/bash
# PMC passes over one kernel (regex) inside bench.py (one field, config 2):
#   bash tools/pmc_kernel.sh <outdir> <kernel regex> [ENV=VAL ...]  (GPU box, repo root)
O=${1:-gpurun_out/pmc_k}; R=${2:-gemm_x6c_kernel}; shift 2
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
K="--kernel-include-regex $R"
B="python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --linear-check 0 ${BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH --kernel-trace -d $O/p1 -o p1 -f csv -- $B > $O/p1.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 $K --pmc GRBM_GUI_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_IFETCH_LEVEL --kernel-trace -d $O/p2 -o p2 -f csv -- $B > $O/p2.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 $K --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d $O/p3 -o p3 -f csv -- $B > $O/p3.txt 2>&1
