set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -m gpu -k "attn or attention" > gpurun_out/r4/g4_attn_pytest.log 2>&1 &&
timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g4_attn_dq2.log 2>&1 &&
DWAMD_ATTN_DQ2=0 timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g4_attn_dq1.log 2>&1 &&
DWAMD_ATTN_DQ2=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -m gpu -k "attn or attention" > gpurun_out/r4/g4_attn_dq2all_pytest.log 2>&1 &&
DWAMD_ATTN_DQ2=2 timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g4_attn_dq2all.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_dkdvw1.so timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g4_attn_dkdvw1.log 2>&1 &&
DWAMD_ATTN_FWD2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -m gpu -k "attn or attention" > gpurun_out/r4/g4_attn_fwd2_pytest.log 2>&1 &&
DWAMD_ATTN_FWD2=1 timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g4_attn_fwd2.log 2>&1 &&
timeout -k 10 400 bash scripts/gpu_attn_pmc128.sh gpurun_out/r4/pmc128 > gpurun_out/r4/g4_pmc.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --model gpt2-1.5b --seq 1024 --micro-batch 8 --steps 6 --storage --ckpt-dir /tmp/dwamd_fsdp_g4 > gpurun_out/r4/g4_fsdp_gpt2_storage.json 2> gpurun_out/r4/g4_fsdp_gpt2_storage.err
