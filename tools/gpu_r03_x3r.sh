# x3r inverse Legendre: parity tests, then an interleaved A/B against the tiled kernel
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_known_answer.py tests/test_gpu_x3h.py tests/test_gpu_config2.py \
  tests/test_gpu_latband.py > gpurun_out/x3r_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/x3r_t.log; exit 1; }
tail -3 gpurun_out/x3r_t.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/x3r_new_$i.log 2>&1 || exit 1
  MSFNO_LEG_X3R=0 timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/x3r_old_$i.log 2>&1 || exit 1
done
for f in gpurun_out/x3r_new_*.log gpurun_out/x3r_old_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage (legendre_inv|legendre_fwd|mlp_fused|transpose_inv) ' $f | awk '{printf "%s=%s ", $3, $4}')"; done
