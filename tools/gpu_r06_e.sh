#!/bin/bash
# A/B, interleaved: where the inner skip runs (persistent skip_hp grid size, CU-masked side
# stream, serial).  Block line only.
set -o pipefail
O=${1:-gpurun_out/r06_e}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
blk() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 \
    --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {l.split()[2]: float(l.split()[3]) for l in open(sys.argv[2]) if " stage " in l}
keys = ["inner_skip", "legendre_fwd", "spectral_prep", "spectral_l0", "transpose_fwd", "mlp_fused"]
print(sys.argv[3], b["value"], b["ms_per_step"], " ".join(f"{k}={st.get(k, 0):.3f}" for k in keys))
PY
}
for i in 1 2; do
  blk def_$i MSFNO_SKIP_GRID=2
  blk g025_$i MSFNO_SKIP_GRID=0.25
  blk g0375_$i MSFNO_SKIP_GRID=0.375
  blk m4_$i MSFNO_SKIP_GRID=0.25 MSFNO_SIDE_CUSTRIDE=4
  blk ser_$i MSFNO_SIDE_STREAM=0
done > $O/summary.txt
cat $O/summary.txt
