set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# steps during a checkpoint flush are ~45 ms slower with a world-1 RCCL
# communicator in the worker (gloo group: no slowdown; standby: no effect)
B="--no-fault --no-frameworks --no-import-fault --out-dir"
DWAMD_BENCH_PG_DESTROY=1 timeout -k 10 300 python bench.py $B gpurun_out/r5/d_destroy > gpurun_out/r5/d_destroy.json 2> gpurun_out/r5/d_destroy.err || exit $?
DWAMD_BENCH_PG_LAZY=1 timeout -k 10 300 python bench.py $B gpurun_out/r5/d_lazy > gpurun_out/r5/d_lazy.json 2> gpurun_out/r5/d_lazy.err || exit $?
TORCH_NCCL_USE_TENSOR_REGISTER_ALLOCATOR_HOOK=0 timeout -k 10 300 python bench.py $B gpurun_out/r5/d_hook0 > gpurun_out/r5/d_hook0.json 2> gpurun_out/r5/d_hook0.err || exit $?
DWAMD_FLUSH_MODE=kernel timeout -k 10 300 python bench.py $B gpurun_out/r5/d_kflush > gpurun_out/r5/d_kflush.json 2> gpurun_out/r5/d_kflush.err || exit $?
echo done
