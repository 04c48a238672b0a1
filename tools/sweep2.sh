# interleaved sweep: each argument a ';'-separated env list ("-" = defaults); two rounds
mkdir -p gpurun_out/sw
for rep in 1 2; do
  for cfg in "$@"; do
    ( IFS=';'; [ "$cfg" != "-" ] && for kv in $cfg; do export "$kv"; done
      timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --stages \
        > gpurun_out/sw/out.json 2> gpurun_out/sw/err.txt ) || { echo "FAILED $cfg"; tail -5 gpurun_out/sw/err.txt; exit 1; }
    v=$(python -c "import json;print(json.load(open('gpurun_out/sw/out.json'))['value'])")
    echo "rep$rep [$cfg] fields/s $v $(grep -E "${SWEEP_GREP:-stage (fft_fwd|inner_skip|mlp_fused) }" gpurun_out/sw/err.txt | awk '{printf "%s=%s ", $3, $4}')"
  done
done
