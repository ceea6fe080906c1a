set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_lazy_zero_gpu.py tests/test_flash_ckpt_gpu.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r4/g24_pytest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r4/g24_smoke.log 2>&1
