#!/bin/bash
# Block orders of the symmetric transposes (MSFNO_TR_XCD = "<fwd><inv>", 0 plain grid,
# 1 m-fastest, 2 latitude-fastest, both XCD-grouped): kernel traces and FETCH_SIZE for
# 00 / 11 / 22, then interleaved block-line pairs 00 vs 22.
set -o pipefail
O=${1:-gpurun_out/r06_af}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_latband.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
for x in 00 11 22; do
  MSFNO_TR_XCD=$x timeout -k 10 200 rocprofv3 --kernel-include-regex transpose --pmc FETCH_SIZE \
    --kernel-trace -d $O/f$x/p -o f -f csv -- python3 bench.py --steps 2 --warmup 1 $ONE \
    > $O/f$x.json 2> $O/f$x.err || exit $?
  for k in transpose_fwd transpose_inv; do echo "== fetch $x $k"; python tools/pmc_summary.py $O/f$x $k; done
  MSFNO_TR_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$x -o kt -- \
    python3 bench.py --steps 20 --warmup 3 $ONE > $O/kt$x.json 2> $O/kt$x.err || exit $?
  find $O/kt$x -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_xcd$x.csv \;
  rm -rf $O/kt$x
done
for i in 1 2 3; do
  for x in 00 22; do
    MSFNO_TR_XCD=$x timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b$x.$i.json 2> $O/b$x.$i.err || exit $?
    echo "XCD=$x $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$x.$i.json)"
  done
done
