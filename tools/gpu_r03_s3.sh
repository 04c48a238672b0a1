set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread tests/test_gpu_x3h.py -m gpu > gpurun_out/s3_x3h.log 2>&1; echo "x3h rc=$?" >> gpurun_out/s3_x3h.log
for t in 7 8; do
  MSFNO_TILES=leg=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config2.py tests/test_gpu_latband.py -m gpu -k "not two_processes" > gpurun_out/s3_leg$t.log 2>&1; echo "rc=$?" >> gpurun_out/s3_leg$t.log
done
for i in 1 2; do
  for t in 1 7 8; do
    MSFNO_TILES=leg=$t timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages > gpurun_out/s3_b${t}_$i.json 2> gpurun_out/s3_b${t}_$i.err || exit 1
  done
done
MSFNO_ENGINE=x3h bash tools/pmc_kernel.sh gpurun_out/pmc_mfh mlp_fused_h_kernel
echo done
