set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 200 python -u scripts/bench_h2d_streams.py > gpurun_out/r4/g25_h2d.jsonl 2>&1
