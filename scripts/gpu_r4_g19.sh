set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 200 python -u scripts/bench_proj_wgrad.py > gpurun_out/r4/g19_proj_wgrad.jsonl 2>&1
