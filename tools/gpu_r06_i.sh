#!/bin/bash
# A/B, interleaved, block line: fused-MLP fragment-read lead (MSFNO_MH_AHEAD) and the side
# stream's priority with the quarter-CU skip grid.
set -o pipefail
O=${1:-gpurun_out/r06_i}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
blk() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 \
    --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {l.split()[2]: float(l.split()[3]) for l in open(sys.argv[2]) if " stage " in l}
keys = ["mlp_fused", "inner_skip", "legendre_fwd", "spectral_l0", "spectral_l1", "spectral_l2"]
print(sys.argv[3], b["value"], b["ms_per_step"], " ".join(f"{k}={st.get(k, 0):.3f}" for k in keys))
PY
}
for i in 1 2; do
  blk a2_$i MSFNO_MH_AHEAD=2
  blk a1_$i MSFNO_MH_AHEAD=1
  blk a3_$i MSFNO_MH_AHEAD=3
  blk pn_$i MSFNO_SIDE_PRIO=normal
done > $O/summary.txt
cat $O/summary.txt
