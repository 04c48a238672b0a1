set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04_v3
# 0. weight-stationary skip vs per-tile skip_h (bitwise)
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_skip_ws.py > gpurun_out/r04_v3/skip_ws.log 2>&1 || exit $?
# 1. linear filter on S vs gathered, side stream on / off (bitwise)
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 360 --timeout-method thread -m gpu \
  tests/test_gpu_linear_direct.py > gpurun_out/r04_v3/lin_direct.log 2>&1
rc=$?; echo "lin_direct rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# 2. PX co-residency: the register-prefetch r2c (no LDS-DMA), and gemm_x3 instead of skip_h
for v in "MSFNO_FFT_DMA=0" "MSFNO_SKIP_H=0"; do
  env $v MSFNO_SKIP_PX=1 MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 300 \
    python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_configs.py -m gpu \
    -k config3_net > gpurun_out/r04_v3/px_${v%%=*}.log 2>&1
  rc=$?
  echo "$v rc $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
# 3. the persistent MLP: tests
MSFNO_MH_PERSIST=1 timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_gpu_mlp_persist.py tests/test_gpu_x3h_range.py tests/test_gpu_mlp_fused.py -m gpu \
  > gpurun_out/r04_v3/hp_tests.log 2>&1
rc=$?; echo "hp tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# 4. benches: default, persistent MLP, per-tile skip
timeout -k 10 300 python bench.py > gpurun_out/r04_v3/bench.json 2> gpurun_out/r04_v3/bench.err || exit $?
MSFNO_MH_PERSIST=1 timeout -k 10 300 python bench.py > gpurun_out/r04_v3/bench_hp.json 2> gpurun_out/r04_v3/bench_hp.err || exit $?
MSFNO_SKIP_WS=0 timeout -k 10 300 python bench.py > gpurun_out/r04_v3/bench_skiph.json 2> gpurun_out/r04_v3/bench_skiph.err || exit $?
cd /tmp && export TMPDIR=/tmp
MSFNO_MH_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r04_v3/prof_hp -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 > /root/repo/gpurun_out/r04_v3/prof_hp.log 2>&1 || exit $?
exit 0
