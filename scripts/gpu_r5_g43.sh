set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# dK/dV at D=64 with 32-query tiles (160 VGPRs, no spills; 64: 168 + 2 spills)
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_bqt32.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -k "attn or attention" > gpurun_out/r5/attn_bqt32_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_base3.log 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_bqt32.so timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_bqt32.log 2>&1 || exit $?
echo done
