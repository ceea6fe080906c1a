set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g21
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the ring-deferral test alone, with the ring state recorded right after the save
timeout -k 10 300 python -u -m pytest tests/test_flash_ckpt_gpu.py -m gpu -v --timeout 120 --timeout-method thread -k "ring_snapshot" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "PASSED|FAILED|AssertionError" $O/pytest.log | head; grep -E "^E " $O/pytest.log | head -5 | cut -c1-600
exit $rc
