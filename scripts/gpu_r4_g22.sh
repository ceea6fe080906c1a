set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run22 > gpurun_out/r4/g22_bench.json 2> gpurun_out/r4/g22_bench.err &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r4/g22_step.log 2>&1
