set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04_v1
# 1. the FFT/skip co-residency check with the LDS waits in the Stockham passes (per-tile MLP)
MSFNO_FFT_OUTDBG=3 MSFNO_MH_PERSIST=0 MSFNO_SKIP_PX=1 MSFNO_PX_CHECK=1 MSFNO_PX_LOG=1 timeout -k 10 300 \
  python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k config3_net > gpurun_out/r04_v1/pxchk_out3.log 2>&1
rc=$?
echo "px rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# 2. the persistent fused MLP: A/B against the per-tile kernel, oracle, range guard
MSFNO_MH_PERSIST=1 timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_gpu_mlp_persist.py tests/test_gpu_x3h_range.py tests/test_gpu_mlp_fused.py -m gpu \
  > gpurun_out/r04_v1/hp_tests.log 2>&1
rc=$?
echo "hp tests rc $rc"
if [ $rc -ne 0 ]; then exit $rc; fi
# 3. bench: persistent vs per-tile
MSFNO_MH_PERSIST=1 timeout -k 10 300 python bench.py > gpurun_out/r04_v1/bench_hp.json 2> gpurun_out/r04_v1/bench_hp.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r04_v1/bench_tile.json 2> gpurun_out/r04_v1/bench_tile.err || exit $?
cd /tmp && export TMPDIR=/tmp
MSFNO_MH_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r04_v1/prof_hp -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 > /root/repo/gpurun_out/r04_v1/prof_hp.log 2>&1 || exit $?
exit 0
