#!/bin/bash
# Side-stream skip grid share (MSFNO_SKIP_GRID, workgroups per CU) after the transpose
# changes: interleaved block-line rounds at 0.21875 / 0.25 / 0.265625 (56 / 64 / 68 CUs).
set -o pipefail
O=${1:-gpurun_out/r06_ah}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
for i in 1 2 3; do
  for g in 0.25 0.21875 0.265625; do
    MSFNO_SKIP_GRID=$g timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b$g.$i.json 2> $O/b$g.$i.err || exit $?
    echo "GRID=$g $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$g.$i.json)"
  done
done
