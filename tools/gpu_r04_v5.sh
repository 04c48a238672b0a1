set -o pipefail
cd /root/repo
O=gpurun_out/r04_v5
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
# 1. the skip kernels serial (side stream off: inner_skip is the kernel's own time) and
#    overlapped, per-tile skip_h vs weight-stationary skip_ws
for cfg in "MSFNO_SIDE_STREAM=0" "MSFNO_SIDE_STREAM=0 MSFNO_SKIP_WS=1" "MSFNO_SKIP_WS=1"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 240 python bench.py --stages --linear-check 0 --cpu-baseline 0 > $O/bench_$tag.json 2> $O/bench_$tag.err || exit $?
done
# 2. does skip_ws corrupt a co-resident forward FFT like skip_h (PX mode, the side
#    kernel at block start = skip with per-channel scales 1 -> skip_ws)?
MSFNO_SKIP_WS=1 MSFNO_SKIP_PX=1 MSFNO_PX_SIDEK=ones MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 200 \
  $T -x --timeout 180 tests/test_gpu_configs.py -k config3_net > $O/px_ws_ones.log 2>&1
rc=$?; echo "px ws rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
# 3. the same with skip_h (reference for the diagnostic)
MSFNO_SKIP_PX=1 MSFNO_PX_SIDEK=ones MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 200 \
  $T -x --timeout 180 tests/test_gpu_configs.py -k config3_net > $O/px_h_ones.log 2>&1
rc=$?; echo "px h rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
exit 0
