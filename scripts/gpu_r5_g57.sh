set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/g57
export HSA_ENABLE_IPC_MODE_LEGACY=0
# final driver-style bench (as the driver runs it: no flags)
timeout -k 10 900 python -u bench.py > gpurun_out/r5/g57/bench.json 2> gpurun_out/r5/g57/bench.err || exit $?
echo done
