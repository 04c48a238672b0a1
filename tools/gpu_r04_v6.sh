set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r04_v6
timeout -k 10 120 ./tools/lds_dma_probe > gpurun_out/r04_v6/lds_dma_probe.log 2>&1 || exit $?
exit 0
