#!/bin/bash
# attention kernel iteration: numerics then timing
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -15 gpurun_out/pytest_attn.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1
rc=$?; echo attn_rc=$rc; grep "{" gpurun_out/attn_bench.log
exit $rc
