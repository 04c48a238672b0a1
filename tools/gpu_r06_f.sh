#!/bin/bash
# (1) fused-MLP per-workgroup trace (MSFNO_MH_TRACE) of a block-line run; (2) A/B of the
# persistent inner-skip grid (workgroups per CU), interleaved.
set -o pipefail
O=${1:-gpurun_out/r06_f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
MSFNO_MH_TRACE=$O/mh.trace timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 \
  --linear-check 0 --net-check 0 > $O/trace_bench.json 2> $O/trace_bench.err || exit $?
python tools/mh_trace.py $O/mh.trace > $O/mh_trace.txt 2>&1 || exit $?
blk() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 \
    --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = {l.split()[2]: float(l.split()[3]) for l in open(sys.argv[2]) if " stage " in l}
keys = ["inner_skip", "legendre_fwd", "spectral_prep", "spectral_l0", "spectral_l1", "mlp_fused"]
print(sys.argv[3], b["value"], b["ms_per_step"], " ".join(f"{k}={st.get(k, 0):.3f}" for k in keys))
PY
}
for i in 1 2 3; do
  for g in 0.1875 0.25 0.3125 2; do blk g${g}_$i MSFNO_SKIP_GRID=$g; done
done > $O/summary.txt
cat $O/mh_trace.txt $O/summary.txt
