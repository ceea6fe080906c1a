#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$name.log; [ $rc -ge 124 ] && exit $rc; return 0; }
run d2h 400 python scripts/bench_d2h.py
DWAMD_FLUSH_CU_STRIDE=8 run bench_cu8_i4 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4
DWAMD_FLUSH_CU_STRIDE=4 run bench_cu4_i4 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4
