set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/prof_fsdp_half
export HSA_ENABLE_IPC_MODE_LEGACY=0
# Llama-3-8B FSDP: bf16 params + fp32 masters, with / without activation checkpointing
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 6 > gpurun_out/r5/fsdp_half_noac.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 6 --act-ckpt on > gpurun_out/r5/fsdp_half_ac.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_fsdp_half -o run -- python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 > gpurun_out/r5/prof_fsdp_half/bench.log 2>&1 || exit $?
find gpurun_out/r5/prof_fsdp_half -name "*kernel_trace*" -delete
# attention D=64 (GPT2 shape) counters with the three-wave dQ
bash scripts/gpu_attn_pmc64.sh gpurun_out/r5/pmc64 || exit $?
echo done
