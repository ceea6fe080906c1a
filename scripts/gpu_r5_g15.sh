set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# reproduced: process group after the model + flush stream after the group
# -> 147 ms/step (flush stream created first: 109).  Which queue is shared?
L=gpurun_out/r5/g15_queues.log
AB="python -u scripts/bench_step_ab.py --steps 20 --variant off --flush-gb 8 --flush-dst shm --pg nccl --pg-late"
DWAMD_FLUSH_STREAM=cumask timeout -k 10 200 $AB >> $L 2>&1 || exit $?
DWAMD_FLUSH_STREAM=plain timeout -k 10 200 $AB >> $L 2>&1 || exit $?
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 200 $AB >> $L 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $AB >> $L 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off --pg nccl --pg-late >> $L 2>&1 || exit $?
echo done
