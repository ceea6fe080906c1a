set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run16 > gpurun_out/r4/g16_bench.json 2> gpurun_out/r4/g16_bench.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hbm_tier_gpu.py tests/test_rehearsal_gpu.py tests/test_lazy_zero_gpu.py -m gpu > gpurun_out/r4/g16_pytest.log 2>&1
