#!/bin/bash
# A/B of runtime switches in the full block: each argument is a list of VAR=value
# assignments separated by ';' (e.g. "MSFNO_SPEC_4M=1;MSFNO_TILES=fc2=0"), one bench per argument.
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  ( IFS=';'; for kv in $cfg; do export "$kv"; done
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --stages \
      > gpurun_out/sweep/out.json 2> gpurun_out/sweep/err.txt ) || { echo "FAILED $cfg"; tail -5 gpurun_out/sweep/err.txt; exit 1; }
  v=$(python -c "import json;print(json.load(open('gpurun_out/sweep/out.json'))['ms_per_step'])")
  echo "== [$cfg] ms/step $v"
  grep -E "${SWEEP_GREP:-mlp_fc|inner_skip|spectral_|legendre}" gpurun_out/sweep/err.txt | tr -s ' ' | sed 's/^/   /'
done
