set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04_v0
# the x3h range guard of the fused MLP, and the MLP parity tests
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_x3h_range.py tests/test_gpu_mlp_fused.py tests/test_gpu_x3h.py -m gpu \
  > gpurun_out/r04_v0/range.log 2>&1 || exit $?
# bench of this build
timeout -k 10 300 python bench.py > gpurun_out/r04_v0/bench.json 2> gpurun_out/r04_v0/bench.err || exit $?
# MSFNO_SKIP_PX ordering diagnostics on the config-3 network (assertion failures are data)
for mode in 1 2 3; do
  MSFNO_SKIP_PX=1 MSFNO_PX_CHECK=$mode timeout -k 10 300 python -u -m pytest -x -v -s \
    --timeout 280 --timeout-method thread tests/test_gpu_configs.py -m gpu -k config3_net \
    > gpurun_out/r04_v0/pxchk_$mode.log 2>&1
  rc=$?
  echo "mode $mode rc $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
