#!/bin/bash
# Round-6 HEAD measurement (GPU box, repo root): full -m gpu suite, smoke, the round
# profile (kernel trace + FETCH/WRITE PMC passes + bench line with stages) and
# MFMA-busy / wait PMC for the block's three largest kernels.
set -o pipefail
O=${1:-gpurun_out/r06_final}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile_round.sh $O || exit $?
for k in mlp_fused_h_kernel legendre_x3f_kernel skip_hp_kernel; do
  timeout -s KILL 120 rocprofv3 --kernel-include-regex $k --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU \
    --kernel-trace -d $O/pmc_$k -o p -f csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 \
    --linear-check 0 --net-check 0 > $O/pmc_$k.txt 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/gpu_suite.log 2>&1; rc=$?; echo "suite rc $rc" >> $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
exit 0
