set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g7
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# import-mode (HBM tier off) stall after every save: which stream shares the queue?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only-import --out-dir $O/v1 > $O/v1.json 2> $O/v1.err || exit $?
DWAMD_DEFER_OPTIM_RESTORE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only-import --out-dir $O/v2 > $O/v2.json 2> $O/v2.err || exit $?
DWAMD_STANDBY_FLUSH_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only-import --out-dir $O/v3 > $O/v3.json 2> $O/v3.err || exit $?
DWAMD_STANDBY_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only-import --out-dir $O/v4 > $O/v4.json 2> $O/v4.err || exit $?
echo done
