set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g20
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# whole GPU suite + smoke after the flat-FSDP / FusedLinear changes, as the driver runs them
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 $O/pytest_gpu_full.log; grep -E "FAILED|ERROR" $O/pytest_gpu_full.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
