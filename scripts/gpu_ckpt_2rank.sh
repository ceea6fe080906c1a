#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_flash_ckpt_gpu.py -m gpu -v -k "ddp or two_rank" --timeout 200 --timeout-method thread > gpurun_out/pytest_ckpt2.log 2>&1
rc=$?; echo rc=$rc; grep -E "PASS|FAIL|assert |Error" gpurun_out/pytest_ckpt2.log | head -20
exit $rc
