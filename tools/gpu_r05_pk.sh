# The packed-FP32 co-execution evidence (profiles/r05_pk/): the rFFT of
# the 120 x 240 blocks beside skip_h / gemm_x3 / nothing, the isolated instruction pair
# beside each synthetic aggressor, and the op_sel sweep.  Build: tools/build_tools.sh
set -o pipefail
cd /root/repo
O=gpurun_out/r05_pk
mkdir -p $O
timeout -k 10 300 ./tools/bin/corun_probe 10 > $O/corun.log 2>&1 || exit $?
timeout -k 10 400 ./tools/bin/pk_opsel_sweep 2 > $O/pk_sweep.log 2>&1 || exit $?
