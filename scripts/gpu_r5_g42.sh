set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_flash_ckpt_gpu.py tests/test_hbm_tier_gpu.py > gpurun_out/r5/g42.log 2>&1
rc=$?; echo rc=$rc; tail -2 gpurun_out/r5/g42.log; exit $rc
