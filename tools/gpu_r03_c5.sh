# config-5 divergence curve (band vs unsharded) under both engines
set -o pipefail
cd /root/repo
for eng in x6 x3h; do
  MSFNO_ENGINE=$eng timeout -k 10 300 python -u -m pytest -x -q -s --timeout 250 --timeout-method thread tests/test_gpu_configs.py -m gpu -k config5 > gpurun_out/c5_$eng.log 2>&1
  echo "rc=$?" >> gpurun_out/c5_$eng.log
done
