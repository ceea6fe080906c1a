#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_c.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench_c.log 2>&1
rc=$?; echo attn_rc=$rc; cat gpurun_out/attn_bench_c.log | grep "{"
exit $rc
