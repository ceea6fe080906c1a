set -o pipefail
cd $GRAFT_REPO_ROOT
export DWAMD_ATTN_DKDV64W=1
bash scripts/gpu_attn_pmc64.sh gpurun_out/r6/g16 && cat gpurun_out/r6/g16/summary.txt
