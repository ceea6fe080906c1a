#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/gemm_shapes.py > gpurun_out/gemm_shapes.log 2>&1
rc=$?; echo gemm_rc=$rc; cat gpurun_out/gemm_shapes.log | grep "{"
[ $rc -ge 124 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_step -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-fault --ckpt-interval 1000 > $GRAFT_REPO_ROOT/gpurun_out/prof_step.log 2>&1
rc=$?; echo prof_rc=$rc
ls -R $GRAFT_REPO_ROOT/gpurun_out/prof_step | head
exit 0
