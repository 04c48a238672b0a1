#!/bin/bash
# Diagnostic (wrong results): the persistent encoder without its addend stream (1), its
# stores (2), its x stream (4), its GELU (8), or with neither HBM stream but the weights
# (7 = no addend, stores, x), against the default, interleaved: which phase sets its time.
set -o pipefail
O=${1:-gpurun_out/r06_r}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
net() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 --net-check 0 \
    > $O/n_$tag.json 2> $O/n_$tag.err || exit $?
  python - $O/n_$tag.json $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("net", sys.argv[2], b["value"], r.get("ms_per_step"), r.get("all_stages_ms", {}).get("mlp_gen"))
PY
}
for i in 1 2; do
  for d in 0 1 2 4 8 6; do net d${d}_$i MSFNO_MG_DIAG=$d; done
done > $O/summary.txt
cat $O/summary.txt
