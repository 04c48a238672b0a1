# A/B of a run-time switch on the headline bench: ab_env.sh VAR=VALUE [reps]
set -e
mkdir -p gpurun_out
kv="$1"; n=${2:-2}
for i in $(seq 1 $n); do
  timeout -k 10 200 python bench.py --stages > gpurun_out/ab_def_$i.log 2>&1
  env $kv timeout -k 10 200 python bench.py --stages > gpurun_out/ab_new_$i.log 2>&1
done
for f in gpurun_out/ab_def_*.log gpurun_out/ab_new_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage (fft_fwd|inner_skip|mlp_fused) ' $f | awk '{printf "%s=%s ", $3, $4}')"; done
