set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
F="tests/test_flash_ckpt_gpu.py::test_gpu_deferred_optimizer_restore_orders_the_first_step"
# bisect the full-suite-only NaN: which earlier file leaves state behind
timeout -k 10 400 $P tests/test_adam_kernel_gpu.py tests/test_amp_gpu.py tests/test_attention_ext_gpu.py tests/test_context_parallel.py tests/test_data.py tests/test_deterministic_gpu.py $F > gpurun_out/r5/g21_a.log 2>&1
rc=$?; echo a_rc=$rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 $P tests/test_deterministic_gpu.py $F > gpurun_out/r5/g21_b.log 2>&1
rc=$?; echo b_rc=$rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 $P tests/test_adam_kernel_gpu.py tests/test_amp_gpu.py tests/test_attention_ext_gpu.py tests/test_context_parallel.py tests/test_data.py $F > gpurun_out/r5/g21_c.log 2>&1
rc=$?; echo c_rc=$rc; [ $rc -le 1 ] || exit $rc
echo done
