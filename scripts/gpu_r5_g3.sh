set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py tests/test_deterministic_gpu.py tests/test_optim_overlap_gpu.py tests/test_ops_gpu.py tests/test_llama.py > gpurun_out/r5/g3_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -le 1 ] || exit $rc
# which part of a world-1 RCCL process group slows the training step
for pg in none nccl nccl_lazy nccl_destroy gloo; do
  timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off --pg $pg >> gpurun_out/r5/g3_step_pg.log 2>&1 || exit $?
done
TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off --pg nccl >> gpurun_out/r5/g3_step_pg.log 2>&1 || exit $?
TORCH_NCCL_USE_TENSOR_REGISTER_ALLOCATOR_HOOK=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off --pg nccl >> gpurun_out/r5/g3_step_pg.log 2>&1 || exit $?
NCCL_RUNTIME_CONNECT=0 RCCL_MSCCL_ENABLE=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off --pg nccl >> gpurun_out/r5/g3_step_pg.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pg in none nccl; do
  mkdir -p gpurun_out/r5/prof_pg_$pg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_pg_$pg -o run -- python3 scripts/bench_step_ab.py --steps 6 --variant off --pg $pg > gpurun_out/r5/prof_pg_$pg/log.txt 2>&1 || exit $?
  find gpurun_out/r5/prof_pg_$pg -name "*kernel_trace*" -delete
done
echo done
