#!/bin/bash
# Parameter gradients (msfno_block_backward_params / msfno_mlp_backward_params) vs fp64
# oracle autograd, then the bench line (block) once.
set -o pipefail
O=${1:-gpurun_out/r06_g}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 500 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_film_backward.py > $O/film_backward.log 2>&1; rc=$?
echo "rc $rc" >> $O/film_backward.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/dma_rate.hip -o $O/dma_rate > $O/dma_rate.txt 2>&1 && \
  timeout -k 10 120 $O/dma_rate >> $O/dma_rate.txt 2>&1; rm -f $O/dma_rate
exit $rc
timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 --linear-check 0 --net-check 0 \
  --stages > $O/bench.json 2> $O/bench_stages.txt || exit $?
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/dma_rate.hip -o $O/dma_rate > $O/dma_rate.txt 2>&1 && \
  timeout -k 10 120 $O/dma_rate >> $O/dma_rate.txt 2>&1; rm -f $O/dma_rate
exit $rc
