#!/bin/bash
# Persistent encoder: the fc1 steps' VALU (GELU conversions) scheduled between their
# MFMAs (sched_group_barrier, MSFNO_MG_SG = VALU per MFMA) vs the compiler's order:
# bitwise test under SG=4, interleaved A/B of the net line.
set -o pipefail
O=${1:-gpurun_out/r06_s}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
MSFNO_MG_SG=4 timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_gen.py -k bitwise > $O/tests_sg4.log 2>&1 || exit $?
net() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 \
    > $O/n_$tag.json 2> $O/n_$tag.err || exit $?
  python - $O/n_$tag.json $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("net", sys.argv[2], b["value"], r.get("ms_per_step"), r.get("all_stages_ms", {}).get("mlp_gen"))
PY
}
for i in 1 2; do
  for sg in 0 2 4 6; do net sg${sg}_$i MSFNO_MG_SG=$sg; done
done > $O/summary.txt
grep -h "differ\|passed\|failed" $O/tests_sg4.log | tail -4
cat $O/summary.txt
