#!/bin/bash
# Llama-3 8B: loss trajectory at two learning rates, then a kernel profile of the step
set -u
mkdir -p gpurun_out/prof_llama
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DWAMD_CKPT_SLOTS=1
for lr in 1e-4 2e-5; do
  timeout -k 10 400 python -u bench.py --model llama3-8b --micro-batch 1 --seq 4096 --steps 12 --warmup 1 --ckpt-interval 100 --no-fault --lr $lr > gpurun_out/llama_lr$lr.log 2>&1
  rc=$?; echo lr=$lr rc=$rc; grep "losses" gpurun_out/llama_lr$lr.log
  [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- \
  python bench.py --model llama3-8b --micro-batch 1 --seq 4096 --steps 3 --warmup 1 --ckpt-interval 100 --no-fault > gpurun_out/prof_llama/bench.log 2>&1
rc=$?; echo prof_rc=$rc
find gpurun_out/prof_llama -name "*stats*"
exit $rc
