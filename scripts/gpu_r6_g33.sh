set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g33
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_flat_fsdp_gpu.py > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/pytest.log | head -20; tail -1 $O/pytest.log; exit $rc
