set -o pipefail
cd /root/repo
O=gpurun_out/r04_v15
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
# persistent MLP: correctness first (block parity goldens, fused-MLP tests, range guard)
MSFNO_MH_PERSIST2=1 timeout -k 10 300 $T -x --timeout 120 tests/test_gpu_mlp_fused.py tests/test_gpu_x3h_range.py \
  tests/test_gpu_config2.py > $O/hp_tests.log 2>&1
rc=$?; echo "hp tests rc $rc"; if [ $rc -ne 0 ]; then exit 0; fi
for i in 1 2; do
  MSFNO_MH_PERSIST2=1 timeout -k 10 240 python bench.py --stages --linear-check 0 --cpu-baseline 0 > $O/bench_hp_$i.json 2> $O/bench_hp_$i.err || exit $?
  timeout -k 10 240 python bench.py --stages --linear-check 0 --cpu-baseline 0 > $O/bench_base_$i.json 2> $O/bench_base_$i.err || exit $?
done
exit 0
