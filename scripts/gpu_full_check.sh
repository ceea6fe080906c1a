#!/bin/bash
# full GPU test suite + default bench + kernel profile of the GPT2-1.5B step
set -u
mkdir -p gpurun_out/prof_gpt2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu_full.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo bench_rc=$rc; grep '^{' gpurun_out/bench_gpt2.log | cut -c1-1500
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- \
  python3 bench.py --steps 4 --warmup 2 --ckpt-interval 100 --no-fault > gpurun_out/prof_gpt2/bench.log 2>&1
rc=$?; echo prof_rc=$rc
# keep the summaries only (a kernel trace of a bench run is >64 MiB, and
# gpurun copies nothing back past that)
find gpurun_out/prof_gpt2 -name "*kernel_trace*" -delete
find gpurun_out/prof_gpt2 -name "*.csv" -size +8M -delete
exit $rc
