set -o pipefail
cd /root/repo
O=gpurun_out/r05_g
mkdir -p $O
MSFNO_MH_EPI16=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/parity_e16.log 2>&1 || { echo "parity e16 failed"; exit 1; }
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
}
for i in 1 2; do
  run g1_$i MSFNO_SKIP_GRID=1
  run e16_$i MSFNO_MH_EPI16=1
  run g05_$i MSFNO_SKIP_GRID=0.5
  run g2_$i MSFNO_SKIP_GRID=2
  run serial_$i MSFNO_SIDE_STREAM=0
  run p0_$i MSFNO_SKIP_P=0
  run st10_$i MSFNO_MH_STAG=10
  run ps10_$i MSFNO_MH_PERSIST2=1 MSFNO_MH_STAG=10
done
exit 0
