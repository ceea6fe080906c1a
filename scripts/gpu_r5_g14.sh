set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
L=gpurun_out/r5/g14_sync_each.log
AB="python -u scripts/bench_step_ab.py --steps 20 --variant off --flush-gb 8 --flush-dst shm --sync-each"
timeout -k 10 200 $AB --pg none >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --pg-late >> $L 2>&1 || exit $?
B="--no-fault --no-frameworks --no-import-fault --out-dir"
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py $B gpurun_out/r5/e_hwq8 > gpurun_out/r5/e_hwq8.json 2> gpurun_out/r5/e_hwq8.err || exit $?
echo done
