set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lazy_zero_gpu.py tests/test_fused_mlp_gpu.py tests/test_norm_fold_gpu.py tests/test_linear_bgrad_gpu.py tests/test_optim_overlap_gpu.py tests/test_ops_gpu.py tests/test_flash_ckpt_gpu.py -m gpu > gpurun_out/r4/g14_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant off > gpurun_out/r4/g14_step.log 2>&1 &&
DWAMD_LAZY_ZERO_GRAD=0 timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant off > gpurun_out/r4/g14_step_eager.log 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run14 > gpurun_out/r4/g14_bench.json 2> gpurun_out/r4/g14_bench.err
