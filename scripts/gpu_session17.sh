#!/bin/bash
# fused residual add+norm, self-cleaning colred workspace
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m pytest tests -m gpu -x -q -k "norm or colsum or direct or gpt2 or attention" > gpurun_out/pytest_gpu17.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu17.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench17.log 2>&1
rc=$?; echo attn_rc=$rc; cat gpurun_out/attn_bench17.log | grep "{"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-fault > gpurun_out/bench17.log 2>&1
rc=$?; echo bench_rc=$rc; grep -o '"train_step_ms": [0-9.]*\|"tokens_per_s": [0-9.]*\|"loss": [0-9.]*' gpurun_out/bench17.log
[ $rc -ge 124 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof17 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-fault > $GRAFT_REPO_ROOT/gpurun_out/prof17.log 2>&1
echo prof_rc=$?
exit 0
