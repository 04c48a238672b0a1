#!/bin/bash
# Diagnostic (wrong results): the spectral hidden layers (x3h, three stages) without
# their epilogue, against the default, interleaved: the epilogue's share of the layer.
set -o pipefail
O=${1:-gpurun_out/r06_t}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
blk() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 --linear-check 0 --net-check 0 \
    --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, re, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = dict(re.findall(r"stage (\w+)\s+([\d.]+) ms", open(sys.argv[2]).read()))
print("blk", sys.argv[3], b["value"], b["ms_per_step"], {k: st[k] for k in ("spectral_l0", "spectral_l1", "spectral_l2", "spectral_out") if k in st})
PY
}
for i in 1 2; do
  blk e_$i
  blk n_$i MSFNO_X3C_DBG8=1
  blk e2_$i MSFNO_SKIP_GRID=2
  blk n2_$i MSFNO_X3C_DBG8=1 MSFNO_SKIP_GRID=2
done > $O/summary.txt
cat $O/summary.txt
