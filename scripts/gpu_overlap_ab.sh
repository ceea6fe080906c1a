#!/bin/bash
# overlapped-snapshot checkpoint: GPU tests, then bench.py with it off / on
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_flash_ckpt_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ckpt_overlap.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "PASS|FAIL|Error" gpurun_out/pytest_ckpt_overlap.log | head -20
[ $rc -ne 0 ] && exit $rc
DWAMD_OVERLAP_SNAPSHOT=0 timeout -k 10 400 python -u bench.py > gpurun_out/bench_blocking.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_overlap.log 2>&1 || exit $?
for f in blocking overlap; do echo $f; grep '^{' gpurun_out/bench_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ['value','save_sec_max','load_sec','load_verified','train_step_ms','ms_per_step','goodput_pct_1fail_per_hour','snapshot']})"; grep "step ms" gpurun_out/bench_$f.log | cut -c1-400; done
