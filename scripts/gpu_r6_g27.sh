set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g27
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# GPU suite + smoke on the current code, then the GPT2-1.5B step kernel table (two-wave norm backward)
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest_gpu_full.log; grep -E "^FAILED" $O/pytest_gpu_full.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 scripts/bench_step_ab.py --steps 6 --variant off > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find $O -name "*kernel_trace*" -delete
grep "{" $O/prof.log | tail -1 | cut -c1-200
