# A/B of run-time variants on one box: correctness of the variant first, then
# interleaved bench runs.  usage: [OLDKV="A=1 B=2"] bash tools/gpu_r03_ab2.sh "VAR=VAL ..." [tests...]
set -o pipefail
cd /root/repo
KV=$1; shift
TESTS=${@:-tests/test_gpu_parity.py tests/test_gpu_config2.py}
env $KV timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS -m gpu > gpurun_out/ab2_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/ab2_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  env $OLDKV timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages > gpurun_out/ab2_old$i.json 2> gpurun_out/ab2_old$i.err || exit 1
  env $KV timeout -k 10 200 python bench.py --cpu-baseline 0 --linear-check 0 --stages > gpurun_out/ab2_new$i.json 2> gpurun_out/ab2_new$i.err || exit 1
done
