# A/B of a fused-MLP switch: ab_mf.sh VAR=VALUE  (bench x2 interleaved + parity with it set)
set -e
mkdir -p gpurun_out
kv="$1"
env $kv timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --stages > gpurun_out/ab_def_$i.log 2>&1
  env $kv timeout -k 10 200 python bench.py --stages > gpurun_out/ab_new_$i.log 2>&1
done
tail -2 gpurun_out/ab_tests.log
for f in gpurun_out/ab_def_[12].log gpurun_out/ab_new_[12].log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage mlp_fused' $f | awk '{print $4}')"; done
