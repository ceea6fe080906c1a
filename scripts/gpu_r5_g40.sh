set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DWAMD_CKPT_SLOTS=1  # one 124 GB shm slot: stays well inside the box's per-command host-memory cap
# Llama-3 70B TP=8 rank shard trained on one GPU, forced 64 GB staging ring:
# the deferred optimizer-state write-back (default) vs waiting for the ring
timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging ring --ring-hbm-gb 64 --ckpt-dir /tmp/r5ring_a > gpurun_out/r5/ring64_defer_b.json 2> gpurun_out/r5/ring64_defer_b.err &&
DWAMD_DEFER_STATE=0 timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging ring --ring-hbm-gb 64 --ckpt-dir /tmp/r5ring_b > gpurun_out/r5/ring64_wait_b.json 2> gpurun_out/r5/ring64_wait_b.err
