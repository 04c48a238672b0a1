#!/bin/bash
# MFMA triples of two tiles / two pixel groups interleaved (no back-to-back accumulator
# dependency): correctness under the switches, then interleaved A/B of the block line
# (MSFNO_MH_DIAG=2) and the net line (MSFNO_MG_ILV=1).
set -o pipefail
O=${1:-gpurun_out/r06_p}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
MSFNO_MH_DIAG=2 MSFNO_MG_ILV=1 timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_gen.py tests/test_gpu_x3h.py tests/test_gpu_mlp_fused.py > $O/tests.log 2>&1 || exit $?
blk() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 --linear-check 0 --net-check 0 \
    --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, re, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = dict(re.findall(r"stage (\w+)\s+([\d.]+) ms", open(sys.argv[2]).read()))
print("blk", sys.argv[3], b["value"], b["ms_per_step"], {k: st[k] for k in ("mlp_fused", "inner_skip") if k in st})
PY
}
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
for i in 1 2 3; do
  blk i0_$i MSFNO_MH_DIAG=0
  blk i1_$i MSFNO_MH_DIAG=2
done > $O/summary.txt
for i in 1 2; do
  net g0_$i MSFNO_MG_ILV=0
  net g1_$i MSFNO_MG_ILV=1
done >> $O/summary.txt
grep -h "passed\|failed" $O/tests.log | tail -3
cat $O/summary.txt
