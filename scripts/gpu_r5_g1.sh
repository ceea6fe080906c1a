set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --out-dir gpurun_out/r5/bench1 > gpurun_out/r5/bench1.json 2> gpurun_out/r5/bench1.err &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_deterministic_gpu.py tests/test_optim_overlap_gpu.py tests/test_flash_ckpt_gpu.py tests/test_ops_gpu.py > gpurun_out/r5/g1_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r5/g1_step_default.log 2>&1 &&
DWAMD_DETERMINISTIC=1 timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r5/g1_step_det.log 2>&1
