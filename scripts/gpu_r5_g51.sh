set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/g51
export HSA_ENABLE_IPC_MODE_LEGACY=0
# save-pause phase breakdown (engine per-phase timers), phase 0 only
DWAMD_CKPT_TIMING=1 timeout -k 10 600 python -u bench.py --no-fault --no-persist --no-frameworks --out-dir gpurun_out/r5/g51/run > gpurun_out/r5/g51/bench.json 2> gpurun_out/r5/g51/bench.err || exit $?
echo done
