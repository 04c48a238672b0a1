#!/bin/bash
# Round profile: kernel-trace stats of bench.py, then separate FETCH_SIZE / WRITE_SIZE PMC passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p2 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p2/kt -o kt -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/p2/bench_kt.json 2> gpurun_out/p2/bench_kt.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/p2/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/p2/bench_f.json 2> gpurun_out/p2/bench_f.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/p2/write -o write -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/p2/bench_w.json 2> gpurun_out/p2/bench_w.err && \
find gpurun_out/p2 -name "*.csv" | xargs ls -la
