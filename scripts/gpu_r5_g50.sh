set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# driver-style 1-GPU bench with the agent's exit watcher
timeout -k 10 900 python -u bench.py > gpurun_out/r5/bench_g50.json 2> gpurun_out/r5/bench_g50.err || exit $?
echo done
