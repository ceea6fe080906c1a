set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $P tests/test_flash_ckpt_gpu.py > gpurun_out/r5/g25_a.log 2>&1
rc=$?; echo a_rc=$rc; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 $P tests/test_flash_ckpt_gpu.py -k "staging_ring or deferred_optimizer_restore_orders" > gpurun_out/r5/g25_b.log 2>&1
rc=$?; echo b_rc=$rc; [ $rc -le 1 ] || exit $rc
echo done
