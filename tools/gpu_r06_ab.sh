#!/bin/bash
# One-launch skip weight prep (sk_prep_kernel): the skip / block / net tests, then a
# kernel trace of the net line.
set -o pipefail
O=${1:-gpurun_out/r06_ab}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_corun.py tests/test_gpu_parity.py tests/test_gpu_x3h.py tests/test_gpu_net.py \
  tests/test_gpu_side_stream.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- \
  python3 bench.py --workload net --steps 20 --warmup 3 --cpu-baseline 0 > $O/kt.json 2> $O/kt.err || exit $?
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_net.csv \;
rm -rf $O/kt
tail -2 $O/tests.log
grep -h "sk_\|chan_affine" $O/kernel_stats_net.csv | cut -c1-160
tail -1 $O/kt.json | cut -c1-200
