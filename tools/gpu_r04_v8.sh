set -o pipefail
cd /root/repo
O=gpurun_out/r04_v8
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
# 0. fused x3h encoder / decoder MLP: accuracy vs fp64 next to x6, then the 73-channel
#    12-block network vs the oracle at 721x1440 and the FiLM backward through the decoder
timeout -k 10 300 $T -x --timeout 200 tests/test_gpu_mlp_gen.py tests/test_gpu_gemm_x6.py > $O/mlp_gen.log 2>&1 || exit $?
timeout -k 10 400 $T -x --timeout 300 tests/test_gpu_configs.py -k "config3 or config5" tests/test_gpu_net.py \
  tests/test_gpu_film_backward.py > $O/net.log 2>&1 || exit $?
# 1. side stream bitwise; band path with the gemm_x3 skip
timeout -k 10 400 $T -x --timeout 200 tests/test_gpu_side_stream.py tests/test_gpu_latband.py > $O/side_band.log 2>&1 || exit $?
# 2. benches: the network (fused enc/dec, then the x6 pair), latband N=1, the block
timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net.json 2> $O/bench_net.err || exit $?
MSFNO_MLP_GEN_H=0 timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net_x6.json 2> $O/bench_net_x6.err || exit $?
timeout -k 10 240 python bench.py --parallel latband --linear-check 0 --cpu-baseline 0 --stages \
  > $O/bench_latband_n1.json 2> $O/bench_latband_n1.err || exit $?
timeout -k 10 240 python bench.py --cpu-baseline 0 --stages > $O/bench.json 2> $O/bench.err || exit $?
exit 0
