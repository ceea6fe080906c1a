#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python scripts/goodput_experiment.py --steps 40 --fail-step 22 --out gpurun_out/goodput_gpt2_1.5b_n1.json > gpurun_out/goodput.log 2>&1
echo rc=$?; tail -1 gpurun_out/goodput.log
