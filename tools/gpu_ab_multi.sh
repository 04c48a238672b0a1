# interleaved A/B/C of run-time switches on the headline bench (stage times on stderr):
# gpu_ab_multi.sh TAG REPS "VAR=V ..." "VAR=V ..." ...   ("-" = defaults)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
tag=$1; reps=$2; shift 2
for i in $(seq 1 $reps); do
  j=0
  for kv in "$@"; do
    j=$((j+1))
    if [ "$kv" = "-" ]; then kv="MSFNO_NOTHING=1"; fi
    env $kv timeout -k 10 200 python bench.py --stages --cpu-baseline 0 --linear-check 0 > gpurun_out/${tag}_c${j}_$i.log 2>&1 || exit 1
  done
done
j=0
for kv in "$@"; do
  j=$((j+1))
  for f in gpurun_out/${tag}_c${j}_*.log; do echo "[$kv] $f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -E 'stage (legendre_inv|legendre_fwd|transpose_fwd|transpose_inv|mlp_fused|inner_skip) ' $f | awk '{printf "%s=%s ", $3, $4}')"; done
done
