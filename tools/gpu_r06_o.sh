#!/bin/bash
# Diagnostic: the block MLP without its GELU (MSFNO_MH_DIAG=1, wrong results) vs with,
# interleaved, to bound what a cheaper GELU could gain.
set -o pipefail
O=${1:-gpurun_out/r06_o}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
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
for i in 1 2; do
  blk g_$i MSFNO_MH_DIAG=0
  blk n_$i MSFNO_MH_DIAG=1
done > $O/summary.txt
cat $O/summary.txt
