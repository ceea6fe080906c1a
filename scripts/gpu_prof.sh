#!/bin/bash
# Kernel-level profile of a short bench run (rocprofv3 kernel trace + stats).
set -u
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PROF_SECS:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-fault ${BENCH_ARGS:-} > gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
# keep the summaries only (a kernel trace of a bench run is >64 MiB)
find gpurun_out/prof -name "*kernel_trace*" -delete
find gpurun_out/prof -name "*.csv" -size +8M -delete
exit $rc
