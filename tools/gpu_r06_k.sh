#!/bin/bash
# Persistent pipelined encoder (mlp_gen_hp_kernel): its tests first (fp64 and bitwise
# against the one-tile-per-workgroup kernel), the network tests, then an interleaved A/B
# of the net line (MSFNO_MG_P=0 vs default) and a kernel trace of the default.
set -o pipefail
O=${1:-gpurun_out/r06_k}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_gen.py > $O/mlp_gen_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_net.py tests/test_gpu_configs.py -k "net or config3 or config5 or rollout" \
  > $O/net_tests.log 2>&1 || exit $?
net() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 \
    > $O/n_$tag.json 2> $O/n_$tag.err || exit $?
  python - $O/n_$tag.json $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("net", sys.argv[2], b["value"], r.get("ms_per_step"), r.get("all_stages_ms", {}))
PY
}
for i in 1 2; do
  net p0_$i MSFNO_MG_P=0
  net p1_$i MSFNO_MG_P=1
done > $O/summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- \
  python3 bench.py --workload net --steps 20 --warmup 3 --cpu-baseline 0 > $O/kt.json 2> $O/kt.err || exit $?
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_net.csv \;
rm -rf $O/kt
cat $O/summary.txt
