#!/bin/bash
# (1) LDS-DMA rate probe (tools/dma_rate.hip, built on the host into tools/probe/);
# (2) A/B, interleaved: MSFNO_MG_EARLY (encoder addend loads issued with x's), net line.
set -o pipefail
O=${1:-gpurun_out/r06_h}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 120 tools/probe/dma_rate > $O/dma_rate.txt 2>&1 || exit $?
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
for i in 1 2 3; do
  net e0_$i MSFNO_MG_EARLY=0
  net e1_$i MSFNO_MG_EARLY=1
done > $O/summary.txt
cat $O/dma_rate.txt $O/summary.txt
