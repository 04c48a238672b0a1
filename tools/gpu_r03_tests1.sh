set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py tests/test_rollout.py tests/test_gpu_net.py -m gpu -k "config4 or linear_block_full or config5_112 or filmed_ecmwf or rollout_of_latband" > gpurun_out/t1.log 2>&1 && timeout -k 10 400 python bench.py > gpurun_out/b1.log 2> gpurun_out/b1.err
