# kernel durations (rocprofv3 kernel trace) of bench.py under x6c diagnostic builds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tdbg
export MSFNO_SIDE_STREAM=0
for d in ${DBGS:-0 6}; do
  MSFNO_X6C_DBG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/tdbg/d$d -o t -f csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/tdbg/d$d.txt 2>&1 || exit 1
done
