set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
# the full-suite prefix that produced the NaN (with diagnostics in the test)
timeout -k 10 600 $P tests/test_adam_kernel_gpu.py tests/test_amp_gpu.py tests/test_attention_ext_gpu.py tests/test_context_parallel.py tests/test_data.py tests/test_deterministic_gpu.py tests/test_flash_ckpt_gpu.py > gpurun_out/r5/g27.log 2>&1
rc=$?; echo rc=$rc; exit $rc
