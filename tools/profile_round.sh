#!/bin/bash
# Round profile (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (kernel durations, rocpd + csv)
#   2. separate FETCH_SIZE and WRITE_SIZE PMC passes (MI355X_MICROARCH.md: one TCC counter group per pass)
#   3. the plain bench line with the CPU baseline
# usage: bash tools/profile_round.sh gpurun_out/<tag>
OUT=${1:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $OUT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/kt -o kt -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $OUT/bench_kt.json 2> $OUT/bench_kt.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $OUT/bench_f.json 2> $OUT/bench_f.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o write -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $OUT/bench_w.json 2> $OUT/bench_w.err && \
timeout -k 10 400 python3 bench.py --stages > $OUT/bench.json 2> $OUT/bench_stages.txt && \
cat $OUT/bench.json
