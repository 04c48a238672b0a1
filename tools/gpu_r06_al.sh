#!/bin/bash
# PMC (issue / LDS / wait counters, three passes each) of the inverse Legendre, the
# transposes and the row FFTs in-block, for what bounds them after round 6.
set -o pipefail
O=${1:-gpurun_out/r06_al}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
# (the row FFTs' row statistics now come from registers, one LDS pass fewer each: parity + timing first)
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_known_answer.py tests/test_gpu_x3h.py tests/test_gpu_large_golden.py tests/test_gpu_net.py tests/test_gpu_configs.py tests/test_gpu_variants.py \
  > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- \
  python3 bench.py --steps 20 --warmup 3 --cpu-baseline 0 --linear-check 0 --net-check 0 > $O/kt.json 2> $O/kt.err || exit $?
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
grep -h "fft_r2c\|fft_c2r" $O/kernel_stats.csv | cut -c1-160
for k in legendre_x3r_kernel legendre_x3f_kernel transpose_fwd_sym4h transpose_inv_sym2 fft_r2c_dma fft_c2r_dma; do
  bash tools/pmc_kernel.sh $O/$k $k > $O/$k.log 2>&1 || exit $?
  echo "== $k"; python tools/pmc_summary.py $O/$k $k | tee $O/$k.txt
  rm -rf $O/$k
done
