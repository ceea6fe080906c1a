set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# Llama-3-8B FSDP2 training with flash checkpoints (bf16 params + fp32 masters, no activation ckpt)
timeout -k 10 500 python -u scripts/bench_fsdp_llama.py --steps 8 --ckpt-interval 4 > gpurun_out/r5/fsdp_llama8b_ckpt.log 2>&1 || exit $?
# Llama-3-70B TP=8 rank shard in Megatron layout (123.5 GB): save pause / restore
DWAMD_CKPT_SLOTS=1 timeout -k 10 600 python -u scripts/bench_megatron_tp_shard.py > gpurun_out/r5/megatron_70b_tp8.log 2>&1 || exit $?
echo done
