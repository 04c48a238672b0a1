set -o pipefail
cd /root/repo
O=gpurun_out/r05_pk_ab
mkdir -p $O
PK=tools/bin/pk/libmsfno.so
timeout -k 10 120 ./tools/bin/corun_probe 5 fft240 > $O/corun_fft240_nopk.log 2>&1 || exit $?
for i in 1 2; do
  for v in nopk pk; do
    if [ $v = pk ]; then export MSFNO_LIB=$PK; else unset MSFNO_LIB; fi
    timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --stages > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || exit $?
    timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 > $O/net_${v}_$i.json 2> $O/net_${v}_$i.err || exit $?
  done
done
unset MSFNO_LIB
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
echo "suite rc $?" >> $O/suite.log
exit 0
