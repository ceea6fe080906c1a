#!/bin/bash
# Restart-after-crash check of the double-buffered shm on the GPU + goodput rerun with diagnostics.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python scripts/ckpt_restart_check.py > gpurun_out/restart_check.log 2>&1
rc=$?; echo restart_rc=$rc; grep -v Warn gpurun_out/restart_check.log | tail -8
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python scripts/goodput_experiment.py --steps 40 --fail-step 22 --out gpurun_out/goodput_gpt2_1.5b_n1.json > gpurun_out/goodput.log 2>&1
rc=$?; echo goodput_rc=$rc; tail -1 gpurun_out/goodput.log
exit 0
