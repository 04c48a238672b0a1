set -o pipefail
cd /root/repo
O=gpurun_out/r04_v13
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
timeout -k 10 500 $T -x --timeout 300 tests/test_gpu_parity.py tests/test_gpu_x3h.py tests/test_gpu_config2.py \
  tests/test_gpu_side_stream.py > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python bench.py --stages --linear-check 0 --cpu-baseline 0 > $O/bench_split_$i.json 2> $O/bench_split_$i.err || exit $?
  MSFNO_SPEC_L0_SPLIT=0 timeout -k 10 240 python bench.py --stages --linear-check 0 --cpu-baseline 0 > $O/bench_f32_$i.json 2> $O/bench_f32_$i.err || exit $?
done
timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net.json 2> $O/bench_net.err || exit $?
exit 0
