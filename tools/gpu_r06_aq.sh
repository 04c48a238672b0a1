#!/bin/bash
# Pass 2 -> 3 of the forward 4 x 4 x ... FFT codelets through an XOR swizzle (the inverse kernel unchanged): parity
# tests, a kernel trace of the block line, three block lines.
set -o pipefail
O=${1:-gpurun_out/r06_aq}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_known_answer.py tests/test_gpu_x3h.py tests/test_gpu_large_golden.py \
  tests/test_gpu_net.py tests/test_gpu_configs.py tests/test_gpu_latband.py tests/test_gpu_variants.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- \
  python3 bench.py --steps 20 --warmup 3 $ONE > $O/kt.json 2> $O/kt.err || exit $?
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats.csv')):
    if 'fft_' in r['Name'] or 'transpose' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])"
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b.$i.json 2> $O/b.$i.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b.$i.json
done
