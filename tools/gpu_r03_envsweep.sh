# one env var over values: bench stage times, interleaved twice.  usage: VAR "v1 v2 ..." [test files]
set -o pipefail
cd /root/repo
VAR=$1; VALS=$2; shift 2
if [ $# -gt 0 ]; then
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread "$@" -m gpu > gpurun_out/sw_t_$v.log 2>&1 || exit 1
  done
fi
for i in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages --steps 10 > gpurun_out/sw_${v}_$i.json 2> gpurun_out/sw_${v}_$i.err || exit 1
  done
done
