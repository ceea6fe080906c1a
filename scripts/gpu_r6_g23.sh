set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g23
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the GPU suite in driver order up to the ring-deferral test (ring state recorded after the save)
timeout -k 10 600 python -u -m pytest tests/test_flash_ckpt_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_flash_ckpt_gpu.py::test_gpu_ring_snapshot_fp32_params_without_master > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; grep -E "^E " $O/pytest.log | head -5 | cut -c1-900
exit 0
