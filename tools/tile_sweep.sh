#!/bin/bash
# A/B of GEMM tile choices per role in the full block (MSFNO_TILES), one bench per config.
# tiles: 0=128x128 1=128x64 3=256x64 4=256x128 5=128x256
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  MSFNO_TILES="$cfg" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --stages \
    > gpurun_out/sweep/out.json 2> gpurun_out/sweep/err.txt || { echo "FAILED $cfg"; tail -5 gpurun_out/sweep/err.txt; exit 1; }
  v=$(python -c "import json;print(json.load(open('gpurun_out/sweep/out.json'))['ms_per_step'])")
  echo "== [$cfg] ms/step $v"
  grep -E "mlp_fc|inner_skip|spectral_|legendre" gpurun_out/sweep/err.txt | tr -s ' ' | sed 's/^/   /'
done
