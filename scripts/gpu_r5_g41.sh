set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_attn_pmc128.sh gpurun_out/r5/pmc128 || exit $?
find gpurun_out/r5/pmc128 -name "*kernel_trace*" -delete
echo done
