#!/bin/bash
set -u
mkdir -p gpurun_out/prof_attn
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 4,4096,32,8,128 > gpurun_out/prof_attn/run.log 2>&1
rc=$?; echo prof_rc=$rc
exit $rc
