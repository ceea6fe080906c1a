#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-1800; [ $rc -ge 124 ] && exit $rc; return 0; }
run build 300 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider
run bench 600 python bench.py
