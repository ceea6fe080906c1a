#!/bin/bash
# TunableOp (hipBLASLt/rocBLAS solution search) for the GPT2-1.5B GEMM shapes.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 12 --warmup 4 --no-fault > gpurun_out/bench_notune.log 2>&1
rc=$?; echo notune_rc=$rc; tail -1 gpurun_out/bench_notune.log | cut -c1-400
[ $rc -ge 124 ] && exit $rc
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=20
timeout -k 10 900 python bench.py --steps 12 --warmup 4 --no-fault > gpurun_out/bench_tune.log 2>&1
rc=$?; echo tune_rc=$rc; tail -1 gpurun_out/bench_tune.log | cut -c1-400
[ $rc -ge 124 ] && exit $rc
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python bench.py --steps 12 --warmup 4 --no-fault > gpurun_out/bench_tuned.log 2>&1
rc=$?; echo tuned_rc=$rc; tail -1 gpurun_out/bench_tuned.log | cut -c1-400
ls -la gpurun_out/tunableop_results* 
exit 0
