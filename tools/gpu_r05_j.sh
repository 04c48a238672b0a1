set -o pipefail
cd /root/repo
O=gpurun_out/r05_j
mkdir -p $O
timeout -k 10 120 tools/bin/dma_rate > $O/dma_rate.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_corun.py tests/test_gpu_parity.py > $O/corun.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 120 python tools/skip_time.py > $O/skip_time.txt 2>&1 || exit $?
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --net-check 0 --stages > $O/b_$tag.json 2> $O/b_$tag.err || exit $?
}
for i in 1 2; do
  run def_$i MSFNO_MH_EPI16=0
  run e16_$i MSFNO_MH_EPI16=1
done
exit 0
