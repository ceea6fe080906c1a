set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="--no-frameworks --no-import-fault --out-dir"
# snapshot copy on the compute stream (default) vs overlapped on a side stream, fenced by the next optimizer step
DWAMD_OVERLAP_SNAPSHOT=1 timeout -k 10 400 python bench.py $B gpurun_out/r5/i_overlap > gpurun_out/r5/i_overlap.json 2> gpurun_out/r5/i_overlap.err || exit $?
timeout -k 10 400 python bench.py $B gpurun_out/r5/i_block > gpurun_out/r5/i_block.json 2> gpurun_out/r5/i_block.err || exit $?
echo done
