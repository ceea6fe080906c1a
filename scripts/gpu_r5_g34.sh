set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/g34
export HSA_ENABLE_IPC_MODE_LEGACY=0
# tests/test_rehearsal_gpu.py[2]'s command, stacks every 45 s
DWAMD_BENCH_STACK_DUMP_S=45 timeout -k 10 330 python -u bench.py --gpus 2 --rehearse-shared-device --model gpt2 --micro-batch 2 --seq 256 --steps 4 --warmup 2 --fault-window 12 --import-window 8 --inject-slow-flush 3 --ckpt-dir /tmp/g34ckpt --timeout 300 --out-dir gpurun_out/r5/g34/run > gpurun_out/r5/g34/out.json 2> gpurun_out/r5/g34/err.log
rc=$?; echo rc=$rc; exit $rc
