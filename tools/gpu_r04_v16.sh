# Validate the unpadded encoder / decoder stream and this round's new A/B switches;
# measure them (interleaved pairs) and trace the network step's kernels
set -o pipefail
cd /root/repo
O=gpurun_out/r04_v16
mkdir -p $O
T="python -u -m pytest -q --timeout-method thread -m gpu"
timeout -k 10 500 $T -x --timeout 200 tests/test_gpu_mlp_gen.py tests/test_gpu_variants.py > $O/tests.log 2>&1 || exit $?
ab() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --cpu-baseline 0 --linear-check 0 $EXTRA > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json;print('$tag', json.loads(open('$O/$tag.json').readline())['value'])" | tee -a $O/summary.txt
}
for i in 1 2; do
  EXTRA="--workload net" ab net_base_$i MSFNO_NONE=1 || exit $?
  EXTRA="--workload net" ab net_gfork_$i MSFNO_GRAPH_FORK=1 || exit $?
  EXTRA="--filter linear" ab lin_base_$i MSFNO_NONE=1 || exit $?
  EXTRA="--filter linear" ab lin_late_$i MSFNO_LIN_SKIP_AT=inv || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_net -o kt -f csv -- python3 bench.py --workload net --cpu-baseline 0 --steps 5 --warmup 2 > $O/kt_net.log 2>&1 || exit $?
exit 0
