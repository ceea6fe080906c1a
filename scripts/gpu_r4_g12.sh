set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_adam_kernel_gpu.py tests/test_ops_gpu.py tests/test_norm_fold_gpu.py tests/test_fused_mlp_gpu.py tests/test_optim_overlap_gpu.py -m gpu > gpurun_out/r4/g12_pytest.log 2>&1 &&
timeout -k 10 120 python -u scripts/bench_norm_fwd.py > gpurun_out/r4/g12_normfwd.jsonl 2>&1 &&
timeout -k 10 120 python -u scripts/bench_norm_fwd.py >> gpurun_out/r4/g12_normfwd.jsonl 2>&1 &&
DWAMD_NORM_FWD_BLOCKS=512 DWAMD_GELU_UNROLL=2 timeout -k 10 120 python -u scripts/bench_norm_fwd.py >> gpurun_out/r4/g12_normfwd.jsonl 2>&1 &&
DWAMD_NORM_FWD_BLOCKS=1024 timeout -k 10 120 python -u scripts/bench_norm_fwd.py >> gpurun_out/r4/g12_normfwd.jsonl 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant off > gpurun_out/r4/g12_step.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant off > gpurun_out/r4/g12_step_old.log 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run12 > gpurun_out/r4/g12_bench.json 2> gpurun_out/r4/g12_bench.err
