set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6/g1
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flash_ckpt_gpu.py tests/test_hbm_tier_gpu.py tests/test_optim_in_backward_gpu.py > gpurun_out/r6/g1/pytest.log 2>&1
echo "pytest rc $?"
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --out-dir gpurun_out/r6/g1/run > gpurun_out/r6/g1/bench.json 2> gpurun_out/r6/g1/bench.err || exit $?
echo done
