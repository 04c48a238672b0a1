set -o pipefail
cd /root/repo
O=gpurun_out/r05_h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_corun.py > $O/corun.log 2>&1 || { echo "corun failed"; exit 1; }
OLD=$PWD/tools/bin/skip5/libmsfno.so
for i in 1 2; do
  timeout -k 10 120 python tools/skip_time.py >> $O/skip_time.txt 2>&1 || exit $?
  MSFNO_LIB=$OLD timeout -k 10 120 python tools/skip_time.py | sed 's/^/skip5 /' >> $O/skip_time.txt 2>&1 || exit $?
done
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
}
for i in 1 2; do
  run new_g1_$i MSFNO_SKIP_GRID=1
  run new_g05_$i MSFNO_SKIP_GRID=0.5
  run new_g2_$i MSFNO_SKIP_GRID=2
  run old_g05_$i MSFNO_SKIP_GRID=0.5 MSFNO_LIB=$OLD
  run old_g2_$i MSFNO_SKIP_GRID=2 MSFNO_LIB=$OLD
  run new_ser_$i MSFNO_SIDE_STREAM=0
  run new_g2e_$i MSFNO_SKIP_GRID=2 MSFNO_MH_EPI16=1
done
exit 0
