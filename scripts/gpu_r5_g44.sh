set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/gpurun_ab/libdw_kernels_ldsacc.so
# norm backward (H < 2048) with LDS column accumulators, one row in flight per wave, 2 blocks per CU
DWAMD_KERNELS_LIB_AB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_lazy_zero_gpu.py tests/test_fused_mlp_gpu.py -k "norm or layer or fold or lazy or mlp or gpt2 or direct" > gpurun_out/r5/ldsacc_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r5/ldsacc_step.log 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$V timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off >> gpurun_out/r5/ldsacc_step.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off >> gpurun_out/r5/ldsacc_step.log 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$V timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off >> gpurun_out/r5/ldsacc_step.log 2>&1 || exit $?
echo done
