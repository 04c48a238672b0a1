set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --stages > gpurun_out/ab_def_$i.log 2>&1
  MSFNO_MF_XS=1 timeout -k 10 200 python bench.py --stages > gpurun_out/ab_new_$i.log 2>&1
done
tail -2 gpurun_out/full_tests.log
for f in gpurun_out/ab_def_[123].log gpurun_out/ab_new_[123].log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage mlp_fused' $f | awk '{print $4}')"; done
