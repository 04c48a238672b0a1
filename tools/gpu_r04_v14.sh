set -o pipefail
cd /root/repo
O=gpurun_out/r04_v14
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout-method thread -m gpu -x --timeout 150 tests/test_gpu_rccl.py > $O/rccl.log 2>&1
echo "rccl rc $?"
exit 0
