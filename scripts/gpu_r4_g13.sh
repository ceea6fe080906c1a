set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u scripts/bench_wgrad_beta.py > gpurun_out/r4/g13_wgrad_beta.jsonl 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run13 > gpurun_out/r4/g13_bench.json 2> gpurun_out/r4/g13_bench.err &&
DWAMD_RESTORE_GC=1 timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run13gc > gpurun_out/r4/g13_bench_gc.json 2> gpurun_out/r4/g13_bench_gc.err
