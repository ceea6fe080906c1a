set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# Llama-3-8B FSDP2 step: reshard_after_forward on (default) vs off (zero2), alternating
for r in off on off on; do
  timeout -k 10 300 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --reshard $r >> gpurun_out/r5/fsdp_reshard_ab.jsonl 2>> gpurun_out/r5/fsdp_reshard_ab.err || exit $?
done
# flash checkpoint of the zero2-wrapped model (save + verified restore)
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --steps 8 --reshard off > gpurun_out/r5/fsdp_zero2_ckpt.json 2> gpurun_out/r5/fsdp_zero2_ckpt.err || exit $?
echo done
