#!/bin/bash
# PMC of the Legendre kernels, the transposes and the row FFTs at config 2 only (no
# network line: its 120x240 launches would dilute the averages).
set -o pipefail
O=${1:-gpurun_out/r06_ao}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
export BENCH_ARGS="--net-check 0"
for k in legendre_x3f_kernel legendre_x3r_kernel transpose_fwd_sym4h transpose_inv_sym2 fft_r2c_dma fft_c2r_dma gemm_x6c_kernel; do
  bash tools/pmc_kernel.sh $O/$k $k > $O/$k.log 2>&1 || exit $?
  python tools/pmc_summary.py $O/$k $k > $O/$k.txt
  echo "== $k"; grep -h "BANK_CONFLICT\|LDS_IDX_ACTIVE\|WAIT_INST_LDS\|WAVE_CYCLES\|duration\|INSTS_LDS\|INSTS_VALU\|MFMA_BUSY\|mfma_busy" $O/$k.txt
  rm -rf $O/$k
done
