set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the whole GPU suite (what the driver runs at round end) + smoke
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/g56_pytest_gpu_all.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r5/g56_pytest_gpu_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/g56_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/r5/g56_smoke.log; exit $rc
