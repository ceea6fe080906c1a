set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u scripts/find_copies.py > gpurun_out/r4/g18_copies.log 2>&1
