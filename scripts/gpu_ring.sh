#!/bin/bash
# ckpt GPU tests, then the 70B TP=8 shard with its model training on the same
# GPU: auto staging (full buffer when it fits) vs the bounded ring
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ring
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_flash_ckpt_gpu.py > gpurun_out/ring/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ring/pytest.log; [ $rc -ne 0 ] && exit $rc
for st in auto ring; do
  DWAMD_CKPT_TIMING=1 timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging $st --steps 21 \
    --ckpt-interval 10 > gpurun_out/ring/tp_shard_$st.log 2>&1
  rc=$?; echo "$st rc=$rc"; grep "^{" gpurun_out/ring/tp_shard_$st.log | cut -c1-3000
  [ $rc -ne 0 ] && exit $rc
done
exit 0
