set -o pipefail
cd /root/repo
O=gpurun_out/r04_v4
mkdir -p $O
T="python -u -m pytest -v -s --timeout-method thread -m gpu"
# 0. weight-stationary skip vs per-tile skip_h (bitwise); stop on failure (it is the default)
timeout -k 10 300 $T -x --timeout 250 tests/test_gpu_skip_ws.py > $O/skip_ws.log 2>&1 || exit $?
# 1. persistent MLP (opt-in): A/B, oracle, range guard
MSFNO_MH_PERSIST=1 timeout -k 10 400 $T --timeout 200 tests/test_gpu_mlp_persist.py \
  tests/test_gpu_x3h_range.py > $O/hp_tests.log 2>&1
rc=$?; echo "hp rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
# 2. linear filter on S vs gathered (bitwise, side stream on / off)
timeout -k 10 300 $T --timeout 280 tests/test_gpu_linear_direct.py > $O/lin_direct.log 2>&1
rc=$?; echo "lin rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
# 3. band path (x3f on the exchange buffer) and the network's replicate mode
timeout -k 10 500 $T --timeout 240 tests/test_gpu_latband.py tests/test_gpu_net.py \
  tests/test_gpu_mlp_fused.py > $O/band_net.log 2>&1
rc=$?; echo "band rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
# 4. PX co-residency: register-prefetch r2c (no LDS-DMA); gemm_x3 instead of skip_h
for v in "MSFNO_FFT_DMA=0" "MSFNO_SKIP_H=0"; do
  env $v MSFNO_SKIP_PX=1 MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 200 $T -x --timeout 180 \
    tests/test_gpu_configs.py -k config3_net > $O/px_${v%%=*}.log 2>&1
  rc=$?; echo "$v rc $rc"; if [ $rc -gt 1 ]; then exit $rc; fi
done
# 5. benches: default; persistent MLP; per-tile skip; 4-wave x3c layers (stages to stderr)
timeout -k 10 240 python bench.py --stages > $O/bench.json 2> $O/bench.err || exit $?
MSFNO_MH_PERSIST=1 timeout -k 10 240 python bench.py --stages --linear-check 0 > $O/bench_hp.json 2> $O/bench_hp.err || exit $?
MSFNO_SKIP_WS=0 timeout -k 10 240 python bench.py --stages --linear-check 0 > $O/bench_skiph.json 2> $O/bench_skiph.err || exit $?
MSFNO_X3C_WAVES=4 timeout -k 10 240 python bench.py --stages --linear-check 0 > $O/bench_x3c4.json 2> $O/bench_x3c4.err || exit $?
exit 0
