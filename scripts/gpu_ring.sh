#!/bin/bash
# 70B TP=8 shard with its model training on the same GPU: auto staging (full
# buffer when it fits) vs the bounded ring, checkpoint every 10 steps
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ring
for st in auto ring; do
  DWAMD_CKPT_TIMING=1 timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging $st --steps 21 \
    --ckpt-interval 10 > gpurun_out/ring/tp_shard_$st.log 2>&1
  rc=$?; echo "$st rc=$rc"; grep "^{" gpurun_out/ring/tp_shard_$st.log | cut -c1-3000
  [ $rc -ne 0 ] && exit $rc
done
exit 0
