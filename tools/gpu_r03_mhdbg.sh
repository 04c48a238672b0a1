# x3h MLP diagnostic timing: MSFNO_MH_DBG 0 (real), 1 (no weight streaming), 2 (no MFMAs), 3 (neither)
set -o pipefail
cd /root/repo
for d in ${DBGS:-0 1 2 3}; do
  MSFNO_MH_DBG=$d timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages --steps 10 > gpurun_out/mhdbg_$d.json 2> gpurun_out/mhdbg_$d.err || exit 1
done
