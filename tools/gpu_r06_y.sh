#!/bin/bash
# Spectral hidden layers on 4 waves of 64 x 64 (MSFNO_X3C_W4=1) against 8 waves of
# 32 x 64: parity under W4=1, then interleaved A/B of the block line.
set -o pipefail
O=${1:-gpurun_out/r06_y}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
MSFNO_X3C_W4=1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_x3h.py tests/test_gpu_config2.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit $?
blk() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 --linear-check 0 --net-check 0 \
    --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
  python - $O/b_$tag.json $O/b_$tag.err $tag <<'PY'
import json, re, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = dict(re.findall(r"stage (\w+)\s+([\d.]+) ms", open(sys.argv[2]).read()))
print("blk", sys.argv[3], b["value"], b["ms_per_step"], {k: st[k] for k in ("spectral_l1", "spectral_l2", "spectral_out") if k in st})
PY
}
for i in 1 2 3; do
  blk w0_$i MSFNO_X3C_W4=0
  blk w1_$i MSFNO_X3C_W4=1
done > $O/summary.txt
tail -2 $O/tests.log
cat $O/summary.txt
