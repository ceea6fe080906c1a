set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_r5_attn.sh || exit $?
bash scripts/gpu_r5_commperf.sh || exit $?
bash scripts/gpu_r5_fsdp.sh || exit $?
echo done
