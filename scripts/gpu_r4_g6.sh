set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run2 > gpurun_out/r4/bench2.json 2> gpurun_out/r4/bench2.err &&
bash scripts/gpu_r4_g5.sh > gpurun_out/r4/g5.log 2>&1 &&
bash scripts/gpu_r4_g3b.sh
