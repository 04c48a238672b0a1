#!/bin/bash
# irfft with 12 waves and the codelet's pass-2 swizzle (MSFNO_C2R_SWZ=1) against the
# 16-wave plain kernel: the variant's parity (block goldens), kernel traces, three
# interleaved block-line pairs.
set -o pipefail
O=${1:-gpurun_out/r06_as}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_variants.py -k "C2R" > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
MSFNO_C2R_SWZ=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_large_golden.py > $O/tests_swz.log 2>&1 || exit $?
tail -1 $O/tests_swz.log
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
for x in 1 0; do
  MSFNO_C2R_SWZ=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$x -o kt -- \
    python3 bench.py --steps 20 --warmup 3 $ONE > $O/kt$x.json 2> $O/kt$x.err || exit $?
  find $O/kt$x -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_swz$x.csv \;
  rm -rf $O/kt$x
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_swz$x.csv')):
    if 'fft_c2r' in r['Name']: print('SWZ=$x', r['Name'][:60], r['AverageNs'])"
done
for i in 1 2 3; do
  for x in 0 1; do
    MSFNO_C2R_SWZ=$x timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b$x.$i.json 2> $O/b$x.$i.err || exit $?
    echo "SWZ=$x $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$x.$i.json)"
  done
done
