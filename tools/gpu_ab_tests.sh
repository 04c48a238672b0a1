# parity tests, then an interleaved A/B of a run-time switch: gpu_ab_tests.sh TAG VAR=VALUE
# (the default build is "new", VAR=VALUE the old behaviour)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
tag=$1; kv=$2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_known_answer.py tests/test_gpu_x3h.py tests/test_gpu_config2.py \
  tests/test_gpu_latband.py > gpurun_out/${tag}_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -3 gpurun_out/${tag}_t.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/${tag}_new_$i.log 2>&1 || exit 1
  env $kv timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/${tag}_old_$i.log 2>&1 || exit 1
done
for f in gpurun_out/${tag}_new_*.log gpurun_out/${tag}_old_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage (legendre_inv|legendre_fwd|transpose_fwd|mlp_fused|inner_skip) ' $f | awk '{printf "%s=%s ", $3, $4}')"; done
MSFNO_SIDE_STREAM=0 timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/${tag}_noside.log 2>&1 || exit 1
grep -E "stage|value" gpurun_out/${tag}_noside.log | head -20
