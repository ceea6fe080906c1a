set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/g53
export HSA_ENABLE_IPC_MODE_LEGACY=0
# slot metadata written by the flush thread: checkpoint GPU tests, then the driver-style bench
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_flash_ckpt_gpu.py tests/test_rehearsal_gpu.py tests/test_hbm_tier_gpu.py tests/test_optim_overlap_gpu.py > gpurun_out/r5/g53/pytest.log 2>&1 || exit $?
DWAMD_CKPT_TIMING=1 timeout -k 10 900 python -u bench.py --out-dir gpurun_out/r5/g53/run > gpurun_out/r5/g53/bench.json 2> gpurun_out/r5/g53/bench.err || exit $?
echo done
