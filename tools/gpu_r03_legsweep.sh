# x3h Legendre variants (tile width x prefetch depth) vs the fp32-MFMA descriptor GEMM
# usage: [EXTRA="ENV=VAL"] [VARIANTS="..."] bash tools/gpu_r03_legsweep.sh
set -o pipefail
cd /root/repo
V=${VARIANTS:-"MSFNO_LEG_X3=0;MSFNO_LEG_X3_BN=64 MSFNO_LEG_X3_PF=1;MSFNO_LEG_X3_BN=64 MSFNO_LEG_X3_PF=2;MSFNO_LEG_X3_BN=192 MSFNO_LEG_X3_PF=1;MSFNO_LEG_X3_BN=192 MSFNO_LEG_X3_PF=2"}
[ -n "$TESTS" ] && { timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread $TESTS -m gpu > gpurun_out/lg_t.log 2>&1 || exit 1; }
IFS=';' read -ra VS <<< "$V"
for i in 1 2; do
  for v in "${VS[@]}"; do
    tag=$(echo $v | tr ' =' '_-')
    env $EXTRA $v timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages --steps 10 > gpurun_out/lg_${tag}_$i.json 2> gpurun_out/lg_${tag}_$i.err || exit 1
  done
done
