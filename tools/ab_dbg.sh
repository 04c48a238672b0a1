# spectral stage times under the x6c diagnostic builds: ab_dbg.sh (GPU box, repo root)
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4}; do
  MSFNO_X6C_DBG=$d timeout -k 10 200 python bench.py --stages --cpu-baseline 0 > gpurun_out/dbg_$d.log 2>&1 || true
  echo "dbg=$d $(grep -E 'stage spectral_(l1|l2|out) ' gpurun_out/dbg_$d.log | awk '{printf "%s=%s ", $3, $4}')"
done
