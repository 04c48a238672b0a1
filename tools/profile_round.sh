#!/bin/bash
# Round profile (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the block line alone (kt), the linear-filter
#      block line (kt_linear) and the 12-block network line (kt_net)
#   2. separate FETCH_SIZE and WRITE_SIZE PMC passes over the same three workloads
#      (MI355X_MICROARCH.md: one TCC counter group per pass)
#   3. the plain bench line (all objects, CPU baseline) with per-stage timings
# usage: bash tools/profile_round.sh gpurun_out/<tag>;  then on the build host
#        python tools/rocpd_summary.py gpurun_out/<tag> profiles/<tag>
OUT=${1:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $OUT || exit 1
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
declare -A W=([""]="" [_linear]="--filter linear" [_net]="--workload net")
for w in "" _linear _net; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/kt$w -o kt -- \
    python3 bench.py --steps 20 --warmup 3 $ONE ${W[$w]} > $OUT/bench_kt$w.json 2> $OUT/bench_kt$w.err || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    p=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $OUT/$p$w -o $p -- \
      python3 bench.py --steps 2 --warmup 1 $ONE ${W[$w]} > $OUT/bench_$p$w.json 2> $OUT/bench_$p$w.err || exit $?
  done
done
timeout -k 10 400 python3 bench.py --stages > $OUT/bench.json 2> $OUT/bench_stages.txt && \
cat $OUT/bench.json
