set -o pipefail
cd /root/repo
O=gpurun_out/r04_v9
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
timeout -k 10 300 $T -x --timeout 200 tests/test_gpu_mlp_gen.py > $O/mlp_gen.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 --stages > $O/bench_net.json 2> $O/bench_net.err || exit $?
# kernel trace of the network step (encoder / decoder kernels separately)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_net -o kt -f csv -- python3 bench.py --workload net --cpu-baseline 0 --steps 5 --warmup 2 > $O/kt_net.log 2>&1 || exit $?
# PMC of the block MLP (MFMA busy / wait-inst of this build)
bash tools/pmc_kernel.sh $O/pmc_mh mlp_fused_h_kernel > $O/pmc_mh.log 2>&1 || exit $?
# PMC of the fused encoder / decoder
BENCH_ARGS="--workload net --graph 0" bash tools/pmc_kernel.sh $O/pmc_mg mlp_gen_h_kernel > $O/pmc_mg.log 2>&1 || exit $?
exit 0
