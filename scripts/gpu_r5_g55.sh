set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/g55
export HSA_ENABLE_IPC_MODE_LEGACY=0
# driver-style bench (metadata written in the pause again), per-phase save timings
DWAMD_CKPT_TIMING=1 timeout -k 10 900 python -u bench.py --out-dir gpurun_out/r5/g55/run > gpurun_out/r5/g55/bench.json 2> gpurun_out/r5/g55/bench.err || exit $?
echo done
