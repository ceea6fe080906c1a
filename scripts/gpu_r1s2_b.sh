#!/bin/bash
# new GPU tests (offload optimizer) + full gpu suite
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -5 gpurun_out/pytest_gpu_b.log
exit $rc
