#!/bin/bash
# Diagnostic (wrong results): the spectral hidden layers (config 2) without the k-loop
# DMA (2), without MFMAs (4), without the k-loop barrier (16), without DMA and barrier
# (18), against the default, interleaved.
set -o pipefail
O=${1:-gpurun_out/r06_aa}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
blk() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 --linear-check 0 --net-check 0 \
    --stages > $O/b_$tag.json 2> $O/b_$tag.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # (the diagnostic builds' output is not finite: rc 1)
  python - $O/b_$tag.err $tag <<'PY'
import re, sys
st = dict(re.findall(r"stage (\w+)\s+([\d.]+) ms", open(sys.argv[1]).read()))
print("blk", sys.argv[2], {k: st[k] for k in ("spectral_l1", "spectral_l2") if k in st})
PY
}
for i in 1 2; do
  for d in 0 2 4 16 18; do blk d${d}_$i MSFNO_X3C_DBG=$d MSFNO_SKIP_GRID=2; done
done > $O/summary.txt
cat $O/summary.txt
