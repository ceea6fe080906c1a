set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g11
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
echo "pytest rc $?"; tail -1 $O/pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --out-dir $O/run > $O/bench.json 2> $O/bench.err || exit $?
echo done
