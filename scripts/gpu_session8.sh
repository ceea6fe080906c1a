#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/bench_d2h.py > gpurun_out/d2h2.log 2>&1; echo rc=$?; tail -1 gpurun_out/d2h2.log
