set -o pipefail
cd /root/repo
O=gpurun_out/r04_v7
mkdir -p $O
T="python -u -m pytest -v --timeout-method thread -m gpu"
timeout -k 10 120 ./tools/lds_dma_probe > $O/lds_dma_probe.log 2>&1 || exit $?
# 0. the changed kernels first (tiled spec<->tril re-layout, band x3f), stop on failure
timeout -k 10 400 $T -x --timeout 200 tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -k "linear or golden or filter_only or batch_consistency" > $O/relayout.log 2>&1 || exit $?
timeout -k 10 300 $T -x --timeout 200 tests/test_gpu_latband.py > $O/latband.log 2>&1 || exit $?
# 1. benches: default (with the linear line), latband N=1, the network step
timeout -k 10 240 python bench.py --stages > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 240 python bench.py --parallel latband --linear-check 0 --cpu-baseline 0 --stages \
  > $O/bench_latband_n1.json 2> $O/bench_latband_n1.err || exit $?
timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net.json 2> $O/bench_net.err || exit $?
# 2. the whole GPU suite
timeout -k 10 600 $T --timeout 200 tests > $O/suite.log 2>&1
echo "suite rc $?"
exit 0
