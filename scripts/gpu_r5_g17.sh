set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="--no-fault --no-frameworks --no-import-fault --out-dir"
# flush stream kind under the agent's GPU_MAX_HW_QUEUES=8, and plain at 4 queues
DWAMD_FLUSH_STREAM=plain timeout -k 10 300 python bench.py $B gpurun_out/r5/f_plain_q8 > gpurun_out/r5/f_plain_q8.json 2> gpurun_out/r5/f_plain_q8.err || exit $?
DWAMD_FLUSH_STREAM=plain DWAMD_GPU_MAX_HW_QUEUES=0 timeout -k 10 300 python bench.py $B gpurun_out/r5/f_plain_q4 > gpurun_out/r5/f_plain_q4.json 2> gpurun_out/r5/f_plain_q4.err || exit $?
DWAMD_GPU_MAX_HW_QUEUES=0 timeout -k 10 300 python bench.py $B gpurun_out/r5/f_lowprio_q4 > gpurun_out/r5/f_lowprio_q4.json 2> gpurun_out/r5/f_lowprio_q4.err || exit $?
echo done
