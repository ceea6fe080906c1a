set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py -k "replay or deferred_state" > gpurun_out/r5/g6_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -le 1 ] || exit $rc
# does a checkpoint flush (D2H into pinned memory on the copier stream) slow
# the training step more when a world-1 RCCL communicator exists?
L=gpurun_out/r5/g6_flush_ab.log
AB="python -u scripts/bench_step_ab.py --steps 20 --variant off --flush-gb 8"
for pg in none nccl gloo; do
  timeout -k 10 200 $AB --pg $pg >> $L 2>&1 || exit $?
done
DWAMD_FLUSH_STREAM=plain timeout -k 10 200 $AB --pg nccl >> $L 2>&1 || exit $?
DWAMD_FLUSH_STREAM=plain timeout -k 10 200 $AB --pg none >> $L 2>&1 || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 200 $AB --pg none >> $L 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $AB --pg nccl >> $L 2>&1 || exit $?
TORCH_NCCL_USE_TENSOR_REGISTER_ALLOCATOR_HOOK=0 timeout -k 10 200 $AB --pg nccl >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl_destroy >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --flusher-first >> $L 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pg in none nccl; do
  d=gpurun_out/r5/prof_flush_$pg
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $d -o run -- python3 scripts/bench_step_ab.py --steps 6 --variant off --flush-gb 8 --pg $pg > $d/log.txt 2>&1 || exit $?
  find $d -name "*kernel_trace*" -delete
done
echo done
