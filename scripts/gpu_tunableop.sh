#!/bin/bash
# PyTorch TunableOp: tune the GPT2-1.5B / Llama-3 8B GEMM shapes on MI355X
# (hipBLASLt + rocBLAS solutions timed per shape), write the results table,
# then re-run the bench using the tuned table only.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=300 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=50
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --no-fault > gpurun_out/tune_gpt2.log 2>&1
rc=$?; echo tune_rc=$rc; tail -2 gpurun_out/tune_gpt2.log | cut -c1-300; ls -la gpurun_out/tunableop_results*.csv
[ $rc -ne 0 ] && exit $rc
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 400 python -u bench.py > gpurun_out/bench_gpt2_tuned.log 2>&1
rc=$?; echo bench_rc=$rc; grep '^{' gpurun_out/bench_gpt2_tuned.log | grep -o '"train_step_ms": [0-9.]*\|"tokens_per_s": [0-9.]*'
exit $rc
