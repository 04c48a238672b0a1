set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --stages > gpurun_out/ab_def_$i.log 2>&1
  MSFNO_X6C_WAVES=4 timeout -k 10 200 python bench.py --stages > gpurun_out/ab_w4_$i.log 2>&1
done
MSFNO_X6C_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config2.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_w4_tests.log 2>&1 || true
for f in gpurun_out/ab_*_[12].log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'spectral_l[012]|spectral_out' $f | awk '{printf "%s=%s ", $3, $4}')"; done
tail -3 gpurun_out/ab_w4_tests.log
