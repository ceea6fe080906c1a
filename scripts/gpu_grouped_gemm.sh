#!/bin/bash
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/gg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_grouped_gemm_gpu.py tests/test_moe.py > gpurun_out/gg/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/gg/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_grouped_gemm.py > gpurun_out/gg/bench.log 2>&1
rc=$?; tail -2 gpurun_out/gg/bench.log; exit $rc
