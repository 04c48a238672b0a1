set -o pipefail
cd /root/repo
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_film_backward.py > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
for i in 1 2; do
  for v in norm0 leg; do
    MSFNO_SKIP_FORK=$v timeout -k 10 200 python bench.py --steps 30 --cpu-baseline 0 --linear-check 0 --net-check 0 --stages > $O/bench_fork_${v}_$i.json 2> $O/bench_fork_${v}_$i.err || exit $?
  done
  for v in 0 1; do
    MSFNO_GRAPH_FORK=$v timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 > $O/net_gfork_${v}_$i.json 2> $O/net_gfork_${v}_$i.err || exit $?
  done
  for v in norm0 inv; do
    MSFNO_LIN_SKIP_AT=$v timeout -k 10 200 python bench.py --filter linear --steps 20 --cpu-baseline 0 --net-check 0 > $O/lin_skip_${v}_$i.json 2> $O/lin_skip_${v}_$i.err || exit $?
  done
done
exit 0
