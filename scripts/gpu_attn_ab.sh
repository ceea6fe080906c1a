#!/bin/bash
# A/B an attention kernel variant selected by an env var: numerics with the
# variant on, then timing off/on.  Usage: gpu_attn_ab.sh VAR
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
VAR=$1
env "$VAR=1" timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/pytest_attn_ab.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_attn_ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_ab_off.log 2>&1 || exit $?
env "$VAR=1" timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_ab_on.log 2>&1 || exit $?
echo OFF; grep "{" gpurun_out/attn_ab_off.log; echo ON; grep "{" gpurun_out/attn_ab_on.log
