set -o pipefail
cd /root/repo
O=gpurun_out/r05_d
mkdir -p $O
MSFNO_BENCH_BACKEND=gloo MSFNO_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err || exit $?
MSFNO_BENCH_BACKEND=gloo MSFNO_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 3 --steps 2 --warmup 1 --replicas-check 0 > $O/bench_n3.json 2> $O/bench_n3.err || exit $?
exit 0
