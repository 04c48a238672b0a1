set -o pipefail
cd /root/repo
O=gpurun_out/r05_a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_corun.py tests/test_gpu_parity.py tests/test_gpu_mlp_gen.py tests/test_gpu_net.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
exit 0
