#!/bin/bash
# Strided/packed attention kernels: numerics, then bench + steady-state kernel profile.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -x -q -k "flash or gpt2" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo attn_tests_rc=$rc; tail -3 gpurun_out/attn_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-fault > gpurun_out/bench15.log 2>&1
rc=$?; echo bench_rc=$rc; grep -o '"train_step_ms": [0-9.]*\|"tokens_per_s": [0-9.]*' gpurun_out/bench15.log
[ $rc -ge 124 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof15 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-fault > $GRAFT_REPO_ROOT/gpurun_out/prof15.log 2>&1
echo prof_rc=$?
exit 0
