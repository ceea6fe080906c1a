set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g5
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# driver-style bench (default queues, import standby's flush stream pre-created)
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --out-dir $O/run > $O/bench.json 2> $O/bench.err || exit $?
# optimizer inside the backward, normal-priority side stream: A/B again
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --optim-in-backward >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
echo done
