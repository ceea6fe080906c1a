#!/bin/bash
# attention numerics + timing, then the Llama-3 70B TP=8 rank-shard Megatron checkpoint bench
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_attn.sh || exit $?
timeout -k 10 700 python -u scripts/bench_megatron_tp_shard.py > gpurun_out/megatron_70b_tp8.log 2>&1
rc=$?; echo megatron_rc=$rc; grep -v "^\[" gpurun_out/megatron_70b_tp8.log | tail -8 | cut -c1-1500
exit $rc
