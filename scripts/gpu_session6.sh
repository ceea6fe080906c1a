#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep "step ms" gpurun_out/$name.log; grep '^{' gpurun_out/$name.log | python3 -c "import sys,json; [print({k:d.get(k) for k in ('value','ms_per_step','train_step_ms','flush_gbps','flush_cus','load_sec','goodput_pct')}) for d in map(json.loads, sys.stdin)]" 2>/dev/null || tail -3 gpurun_out/$name.log; [ $rc -ge 124 ] && exit $rc; return 0; }
run build 300 python -c "import __graft_entry__ as g; g.build()"
DWAMD_FLUSH_STREAM=cumask run A_cumask_cstream 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_STREAM=lowprio run B_lowprio_cstream 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_STREAM=lowprio DWAMD_COMPUTE_STREAM=0 run C_lowprio_null 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_STREAM=highprio run D_highprio_cstream 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
DWAMD_FLUSH_STREAM=plain run E_plain_cstream 600 python bench.py --steps 12 --warmup 4 --ckpt-interval 4 --no-fault
