set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u scripts/debug_deferred_nan.py > gpurun_out/r5/g20_debug_default.log 2>&1; echo rc=$?
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_o3off.so timeout -k 10 120 python -u scripts/debug_deferred_nan.py > gpurun_out/r5/g20_debug_o3off.log 2>&1; echo rc=$?
DWAMD_DEFER_OPTIM_RESTORE=0 timeout -k 10 120 python -u scripts/debug_deferred_nan.py > gpurun_out/r5/g20_debug_nodefer.log 2>&1; echo rc=$?
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py -k "deferred_optimizer_restore_orders" > gpurun_out/r5/g20_pytest.log 2>&1; echo rc=$?
