set -o pipefail
cd /root/repo
O=gpurun_out/r04_v12
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
timeout -k 10 500 $T -x --timeout 300 tests/test_gpu_parity.py tests/test_gpu_net.py tests/test_gpu_mlp_gen.py \
  tests/test_gpu_x3h.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 $T -x --timeout 300 tests/test_gpu_configs.py -k "config3" > $O/config3.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net.json 2> $O/bench_net.err || exit $?
MSFNO_X3C_BM64=0 timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net_bm128.json 2> $O/bench_net_bm128.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_net -o kt -f csv -- python3 bench.py --workload net --cpu-baseline 0 --steps 5 --warmup 2 > $O/kt_net.log 2>&1 || exit $?
exit 0
