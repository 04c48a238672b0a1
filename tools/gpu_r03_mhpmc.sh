# x3h MLP: diagnostic variants + PMC of NG=1 and NG=2
set -o pipefail
cd /root/repo
DBGS="5 6" bash tools/gpu_r03_mhdbg.sh || exit 1
bash tools/pmc_kernel.sh gpurun_out/pmc_mh1 mlp_fused_h_kernel || exit 1
bash tools/pmc_kernel.sh gpurun_out/pmc_mh2 mlp_fused_h_kernel MSFNO_MH_NG=2
