set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g8
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# driver-style bench: deferred optimizer restore on the flush stream
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --out-dir $O/run > $O/bench.json 2> $O/bench.err || exit $?
echo done
