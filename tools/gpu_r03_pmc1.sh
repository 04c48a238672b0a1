set -o pipefail
cd /root/repo
bash tools/pmc_kernel.sh gpurun_out/pmc_mf2 mlp_fused2_kernel && \
bash tools/pmc_kernel.sh gpurun_out/pmc_mf1 mlp_fused_kernel MSFNO_MF2=0 && \
bash tools/pmc_kernel.sh gpurun_out/pmc_leg gemm_f32_kernel && \
echo done
