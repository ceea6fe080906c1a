set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# RCCL communicator init (even destroyed again) slows the steps during a
# checkpoint flush into hipHostRegister'ed shm; a torch-pinned destination
# showed nothing.  Destination kind x process group x registration order.
L=gpurun_out/r5/g12_flush_shm.log
AB="python -u scripts/bench_step_ab.py --steps 20 --variant off --flush-gb 8"
timeout -k 10 200 $AB --pg none --flush-dst shm >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --flush-dst shm >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --flush-dst shm --flusher-first >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --flush-dst pinned >> $L 2>&1 || exit $?
echo done
B="--no-fault --no-frameworks --no-import-fault --out-dir"
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 300 python bench.py $B gpurun_out/r5/e_noreclaim > gpurun_out/r5/e_noreclaim.json 2> gpurun_out/r5/e_noreclaim.err || exit $?
echo done2
