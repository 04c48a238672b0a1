set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04_v2
# 1. where the persistent MLP differs from the per-tile kernel
timeout -k 10 400 python -u tools/hp_diag.py > gpurun_out/r04_v2/hp_diag.log 2>&1
echo "diag rc $?"
# 2. the linear filter on S (no gather / scatter): goldens, C=256 blocks, full-grid properties
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "linear or golden or filter_only or batch_consistency" \
  > gpurun_out/r04_v2/linear_tests.log 2>&1 || exit $?
# 3. bench (config 2 + the linear sub-line)
timeout -k 10 300 python bench.py > gpurun_out/r04_v2/bench.json 2> gpurun_out/r04_v2/bench.err || exit $?
# 4. PX co-residency: the register-prefetch r2c (no LDS-DMA), and gemm_x3 instead of skip_h
for v in "MSFNO_FFT_DMA=0" "MSFNO_SKIP_H=0"; do
  env $v MSFNO_MH_PERSIST=0 MSFNO_SKIP_PX=1 MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 300 \
    python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_configs.py -m gpu \
    -k config3_net > gpurun_out/r04_v2/px_${v%%=*}.log 2>&1
  rc=$?
  echo "$v rc $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
