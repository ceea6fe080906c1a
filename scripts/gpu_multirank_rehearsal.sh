#!/bin/bash
# Rehearse the multi-rank bench path (FlatDDP, 1/L checkpoint slices, gathered
# restore, fault re-formation) with 2 ranks sharing the single GPU over gloo.
# (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's.)
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DWAMD_BENCH_DEVICE=0 DWAMD_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --model gpt2-medium --steps 8 --warmup 2 --micro-batch 4 > gpurun_out/rehearsal_n2.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/rehearsal_n2.log | cut -c1-1500; tail -5 gpurun_out/rehearsal_n2.log | cut -c1-300
exit $rc
