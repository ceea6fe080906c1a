#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/$name.log | python3 -c "import sys,json; [print({k:d.get(k) for k in ('value','ms_per_step','train_step_ms','flush_gbps','flush_cus','flush_mode','load_sec','goodput_pct')}) for d in map(json.loads, sys.stdin)]" 2>/dev/null || tail -3 gpurun_out/$name.log; [ $rc -ge 124 ] && exit $rc; return 0; }
DWAMD_FLUSH_CU_STRIDE=8 run A_cu8_memcpy 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_CU_STRIDE=8 DWAMD_FLUSH_MODE=kernel run B_cu8_kernel 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_CU_STRIDE=1 DWAMD_FLUSH_MODE=kernel DWAMD_FLUSH_BLOCKS=32 run C_plain_kernel32 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
run d2h 400 python scripts/bench_d2h.py
tail -1 gpurun_out/d2h.log
