set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g23_attn_base.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_diagskip.so timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g23_attn_diagskip.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_diagskip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -m gpu -k "attn or attention" > gpurun_out/r4/g23_pytest.log 2>&1 &&
timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g23_attn_base2.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_diagskip.so timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g23_attn_diagskip2.log 2>&1
