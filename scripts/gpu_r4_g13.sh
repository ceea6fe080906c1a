set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py tests/test_optim_overlap_gpu.py tests/test_hbm_tier_gpu.py -m gpu > gpurun_out/r4/g13_pytest.log 2>&1 &&
timeout -k 10 120 python -u scripts/bench_wgrad_beta.py > gpurun_out/r4/g13_wgrad_beta.jsonl 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run13 > gpurun_out/r4/g13_bench.json 2> gpurun_out/r4/g13_bench.err &&
DWAMD_DEFER_OPTIM_RESTORE=0 timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run13nd > gpurun_out/r4/g13_bench_nodefer.json 2> gpurun_out/r4/g13_bench_nodefer.err
