set -o pipefail
cd /root/repo
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_film_backward.py -k "multi_layer" > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
exit 0
