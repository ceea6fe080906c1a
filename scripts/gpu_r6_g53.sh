set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g53
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# whole GPU suite + smoke + the driver's default bench on the current code
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_gpu_full.log; grep -E "^FAILED" $O/pytest_gpu_full.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
