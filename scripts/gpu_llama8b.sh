#!/bin/bash
# Llama-3 8B full training step + flash checkpoint on ONE MI355X (288 GB HBM):
# bf16 weights/grads + fp32 master/Adam in flat buffers, 112 GB checkpoint
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DWAMD_CKPT_SLOTS=1
free -g | head -2
timeout -k 10 900 python -u bench.py --model llama3-8b --micro-batch 1 --seq 4096 --steps 16 --warmup 2 --ckpt-interval 8 --no-fault > gpurun_out/bench_llama8b.log 2>&1
rc=$?; echo bench_rc=$rc; tail -5 gpurun_out/bench_llama8b.log | cut -c1-2000
[ $rc -ne 0 ] && exit $rc
unset DWAMD_CKPT_SLOTS
timeout -k 10 400 python -u bench.py > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo gpt2_rc=$rc; grep '^{' gpurun_out/bench_gpt2.log | cut -c1-1500
exit $rc
