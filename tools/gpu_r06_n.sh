#!/bin/bash
# Raw-buffer addressing of the fused MLP kernels: bitwise test against 64-bit addressing,
# the MLP tests, then interleaved A/B of the block line (MSFNO_MH_BUF) and the net line
# (MSFNO_MG_BUF).
set -o pipefail
O=${1:-gpurun_out/r06_n}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_buf_addressing.py tests/test_gpu_mlp_gen.py tests/test_gpu_x3h_range.py \
  tests/test_gpu_mlp_fused.py > $O/tests.log 2>&1 || exit $?
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
  blk m0_$i MSFNO_MH_BUF=0
  blk m1_$i MSFNO_MH_BUF=1
done > $O/summary.txt
for i in 1 2; do
  net g0_$i MSFNO_MG_BUF=0 MSFNO_MH_BUF=0
  net g1_$i MSFNO_MG_BUF=1 MSFNO_MH_BUF=1
done >> $O/summary.txt
grep -h "differ\|passed\|failed" $O/tests.log | tail -12
cat $O/summary.txt
