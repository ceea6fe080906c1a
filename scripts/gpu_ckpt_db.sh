#!/bin/bash
# double-buffered HBM staging: flash-ckpt GPU tests + headline bench
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_flash_ckpt_gpu.py tests/test_offload_optim.py tests/test_hf_attention.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ckpt_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_ckpt_gpu.log
[ $rc -ne 0 ] && exit $rc
DWAMD_CKPT_TIMING=1 timeout -k 10 400 python -u bench.py > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo bench_rc=$rc; grep "save ms\|save phases" gpurun_out/bench_gpt2.log | cut -c1-250; grep '^{' gpurun_out/bench_gpt2.log | cut -c1-1500
exit $rc
