set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the driver's bench with every round-5 fix, run logs kept
timeout -k 10 1000 python bench.py --out-dir gpurun_out/r5/bench39 > gpurun_out/r5/bench39.json 2> gpurun_out/r5/bench39.err
rc=$?; echo bench_rc=$rc; exit $rc
