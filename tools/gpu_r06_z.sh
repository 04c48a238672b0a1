#!/bin/bash
# PMC of the row FFT kernels in-block: waits, VALU / LDS instruction mix, bank conflicts.
set -o pipefail
O=${1:-gpurun_out/r06_z}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-include-regex 'fft_' --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE --kernel-trace -d $O/pmc_raw -o p -f csv -- python3 bench.py --steps 2 --warmup 1 \
  --cpu-baseline 0 --linear-check 0 --net-check 0 > $O/pmc.json 2>&1 || exit $?
mkdir -p $O/pm/a && find $O/pmc_raw -name "*.csv" -exec mv {} $O/pm/a/ \; && \
python tools/pmc_summary.py $O/pm "fft_c2r" > $O/pmc_fft_c2r.txt 2>&1; \
python tools/pmc_summary.py $O/pm "fft_r2c" > $O/pmc_fft_r2c.txt 2>&1; rm -rf $O/pmc_raw $O/pm
cat $O/pmc_fft_c2r.txt $O/pmc_fft_r2c.txt
