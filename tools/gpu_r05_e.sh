set -o pipefail
cd /root/repo
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_corun.py > $O/corun.log 2>&1 || { echo "corun rc $?"; exit 1; }
for i in 1 2; do
  MSFNO_SKIP_P=0 timeout -k 10 120 python tools/skip_time.py >> $O/skip_time.txt 2>&1 || exit $?
  MSFNO_SKIP_P=1 timeout -k 10 120 python tools/skip_time.py >> $O/skip_time.txt 2>&1 || exit $?
done
for i in 1 2; do
  for v in 0 1; do
    MSFNO_SKIP_P=$v timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --net-check 0 --stages > $O/bench_p${v}_$i.json 2> $O/bench_p${v}_$i.err || exit $?
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/parity.log 2>&1
echo "parity rc $?" >> $O/parity.log
exit 0
