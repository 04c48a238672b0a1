#!/bin/bash
# Spectral layer 0 on 64-row tiles for the small grids (MSFNO_X3C_L0_BM64=1): parity
# under it (goldens, net, config 3), then interleaved A/B of the net line.
set -o pipefail
O=${1:-gpurun_out/r06_ac}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
MSFNO_X3C_L0_BM64=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_net.py tests/test_gpu_configs.py -k "not config5_112" \
  > $O/tests.log 2>&1 || exit $?
net() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 \
    > $O/n_$tag.json 2> $O/n_$tag.err || exit $?
  python - $O/n_$tag.json $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("net", sys.argv[2], b["value"], r.get("ms_per_step"), r.get("all_stages_ms", {}).get("spectral_l0"))
PY
}
for i in 1 2 3; do
  net l0_$i MSFNO_X3C_L0_BM64=0
  net l1_$i MSFNO_X3C_L0_BM64=1
done > $O/summary.txt
tail -2 $O/tests.log
cat $O/summary.txt
