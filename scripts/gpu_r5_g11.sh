set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# dQ with the row constants as an augmented MFMA k-step (-DDWAMD_DQ_AUG=1)
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_aug.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -k "attn or attention" > gpurun_out/r5/attn_aug_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_base2.log 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_aug.so timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_aug.log 2>&1 || exit $?
echo done
