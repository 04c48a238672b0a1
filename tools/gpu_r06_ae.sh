#!/bin/bash
# XCD-grouped block order of the two symmetric transposes (MSFNO_TR_XCD): the spectral /
# band / net parity tests, FETCH_SIZE of the transposes with the order on and off, and
# interleaved block-line pairs.
set -o pipefail
O=${1:-gpurun_out/r06_ae}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_x3h.py tests/test_gpu_latband.py tests/test_gpu_rccl.py \
  tests/test_gpu_large_golden.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
for x in 1 0; do
  MSFNO_TR_XCD=$x timeout -k 10 200 rocprofv3 --kernel-include-regex transpose --pmc FETCH_SIZE \
    --kernel-trace -d $O/f$x -o f -f csv -- python3 bench.py --steps 2 --warmup 1 $ONE \
    > $O/f$x.json 2> $O/f$x.err || exit $?
  echo "== fetch XCD=$x"; python tools/pmc_summary.py $O/f$x transpose_fwd; python tools/pmc_summary.py $O/f$x transpose_inv
  MSFNO_TR_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$x -o kt -- \
    python3 bench.py --steps 20 --warmup 3 $ONE > $O/kt$x.json 2> $O/kt$x.err || exit $?
  find $O/kt$x -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_xcd$x.csv \;
  rm -rf $O/kt$x $O/f$x
  echo "== kt XCD=$x"; grep -h "transpose" $O/kernel_stats_xcd$x.csv | cut -c1-140
done
for i in 1 2 3; do
  for x in 0 1; do
    MSFNO_TR_XCD=$x timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b$x.$i.json 2> $O/b$x.$i.err || exit $?
    echo "XCD=$x $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$x.$i.json)"
  done
done
