#!/bin/bash
# GPT2-1.5B headline bench + Llama-3 8B single-GPU bench (new attention kernels)
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench.py > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo gpt2_rc=$rc; grep '^{' gpurun_out/bench_gpt2.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
DWAMD_CKPT_SLOTS=1 timeout -k 10 600 python -u bench.py --model llama3-8b --micro-batch 1 --seq 4096 --steps 16 --warmup 2 --ckpt-interval 8 --no-fault --lr 2e-5 > gpurun_out/bench_llama8b.log 2>&1
rc=$?; echo llama_rc=$rc; grep '^{\|losses' gpurun_out/bench_llama8b.log | cut -c1-1500
exit $rc
