#!/bin/bash
# PMC of the spectral hidden layer (gemm_x6c x3h, three stages) in-block: MFMA busy,
# waits, LDS instructions, bank conflicts and LDS-array cycles.
set -o pipefail
O=${1:-gpurun_out/r06_w}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
k='gemm_x6c_kernel<true, 4, 2, false, 0, 3, 2, 3'
timeout -s KILL 120 rocprofv3 --kernel-include-regex 'gemm_x6c_kernel' --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE --kernel-trace -d $O/pmc_raw -o p -f csv -- python3 bench.py --steps 2 --warmup 1 \
  --cpu-baseline 0 --linear-check 0 --net-check 0 > $O/pmc.json 2>&1 || exit $?
mkdir -p $O/pm/a && find $O/pmc_raw -name "*.csv" -exec mv {} $O/pm/a/ \; && \
python tools/pmc_summary.py $O/pm "$k" > $O/pmc_x3c_hidden.txt 2>&1; \
python tools/pmc_summary.py $O/pm "gemm_x6c_kernel<false" > $O/pmc_x3c_out.txt 2>&1; rm -rf $O/pmc_raw $O/pm
cat $O/pmc_x3c_hidden.txt $O/pmc_x3c_out.txt
