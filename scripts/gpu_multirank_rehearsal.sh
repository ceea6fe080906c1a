#!/bin/bash
# Rehearse the multi-rank bench path (FlatDDP, 1/L checkpoint slices, gathered
# restore, fault re-formation) with 2 ranks sharing the single GPU over gloo.
# (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the driver's.)
# NPROC=4: gloo's ring all-reduce accumulates in a rank-dependent order, so
# bf16 replicas may differ in the last bit beyond 2 ranks ("replicas_identical":
# false) -- RCCL's reduce-scatter + all-gather hands every rank the same sums.
# Measured: NPROC=2 and 4 both restore verified (load_verified true).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DWAMD_BENCH_DEVICE=0 DWAMD_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus ${NPROC:-2} --model gpt2-medium --steps 8 --warmup 2 --micro-batch 4 > gpurun_out/rehearsal_n${NPROC:-2}.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/rehearsal_n${NPROC:-2}.log | cut -c1-1500; tail -5 gpurun_out/rehearsal_n${NPROC:-2}.log | cut -c1-300
exit $rc
