#!/bin/bash
# Same-box A/B of two builds (MSFNO_LIB): libmsfno_ab.so = HEAD 8cde0b6, libmsfno.so = the
# first FFT pass storing its 16-B halves alternately by lane octet: kernel traces, three
# interleaved block-line pairs.
set -o pipefail
O=${1:-gpurun_out/r06_at}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
AB=$GRAFT_REPO_ROOT/modulated-spherical-fourier-neural-operator_amd/msfno_amd/libmsfno_ab.so
ONE="--cpu-baseline 0 --linear-check 0 --net-check 0"
for v in head ab; do
  if [ $v = ab ]; then export MSFNO_LIB=$AB; else unset MSFNO_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$v -o kt -- \
    python3 bench.py --steps 20 --warmup 3 $ONE > $O/kt$v.json 2> $O/kt$v.err || exit $?
  find $O/kt$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
  rm -rf $O/kt$v
  python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats_$v.csv')):
    if 'fft_' in r['Name']: print('$v', r['Name'][:60], r['AverageNs'])"
done
for i in 1 2 3; do
  for v in ab head; do
    if [ $v = ab ]; then export MSFNO_LIB=$AB; else unset MSFNO_LIB; fi
    timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 $ONE > $O/b$v.$i.json 2> $O/b$v.$i.err || exit $?
    echo "$v $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $O/b$v.$i.json)"
  done
done
