#!/bin/bash
# full GPU suite + smoke + GPT2 bench + kernel profile, then the 70B TP=8 rank-shard checkpoint bench
set -u
bash scripts/gpu_full_check.sh || exit $?
timeout -k 10 700 python -u scripts/bench_megatron_tp_shard.py > gpurun_out/megatron_70b_tp8.log 2>&1
rc=$?; echo megatron_rc=$rc; grep -v "^\[" gpurun_out/megatron_70b_tp8.log | tail -8 | cut -c1-1500
exit $rc
