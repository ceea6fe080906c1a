#!/bin/bash
# GPU tests (incl. FSDP2/DCP), goodput experiment with double-buffered shm + warm standby, bench.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python scripts/goodput_experiment.py --steps 40 --fail-step 22 --out gpurun_out/goodput_gpt2_1.5b_n1.json > gpurun_out/goodput.log 2>&1
rc=$?; echo goodput_rc=$rc; tail -1 gpurun_out/goodput.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/bench.log
exit 0
