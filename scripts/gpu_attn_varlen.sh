#!/bin/bash
# varlen / padded attention numerics + the HF padded batch, then the dense attention suite
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/varlen
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_hf_attention.py -k "attention or padded" > gpurun_out/varlen/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/varlen/pytest.log; exit $rc
