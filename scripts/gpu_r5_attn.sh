set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# dQ variants (attn_bwd.hip macros): A = -DDWAMD_DQ64_O3=1: D=64 dQ with no split tile body, no row-constant
# accumulator init, compiled for 3 waves/SIMD (166 VGPRs, no spills); C = no split (occ 2)
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_dqA.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -k "attn or attention" > gpurun_out/r5/attn_dqA_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_base.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_dqA.so timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_dqA.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_dqC.so timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r5/attn_dqC.log 2>&1
