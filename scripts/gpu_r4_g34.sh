set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
bash scripts/gpu_r4_g4.sh && bash scripts/gpu_r4_g3.sh
