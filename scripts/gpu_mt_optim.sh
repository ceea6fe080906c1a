#!/bin/bash
# Multi-tensor fused optimizer: GPU numerics tests, then Llama-3 8B FSDP2 step
# time through auto_accelerate (torch AdamW vs the multi-tensor kernel, amp vs
# half precision), then a kernel profile of the fused half run.
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_multi_tensor_optim.py > gpurun_out/mt/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/mt/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "amp --torch-optim" "amp" "half"; do
  tag=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --model llama3-8b --seq 4096 --steps 6 --no-ckpt \
    --precision $cfg > gpurun_out/mt/llama_$tag.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; tail -1 gpurun_out/mt/llama_$tag.log
  [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mt/prof -o run -- \
  python scripts/bench_fsdp_llama.py --model llama3-8b --seq 4096 --steps 3 --no-ckpt --precision half \
  > gpurun_out/mt/prof.log 2>&1
rc=$?; echo prof_rc=$rc
exit $rc
