set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlp_fused.py tests/test_gpu_parity.py tests/test_gpu_config2.py -m gpu > gpurun_out/mf2_t.log 2>&1
echo "tests rc=$?" >> gpurun_out/mf2_t.log
for i in 1 2; do
  MSFNO_MF2=0 timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages > gpurun_out/mf2_old$i.json 2> gpurun_out/mf2_old$i.err || exit 1
  timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages > gpurun_out/mf2_new$i.json 2> gpurun_out/mf2_new$i.err || exit 1
done
