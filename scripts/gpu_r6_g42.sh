set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g42
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# Llama-3-8B step on the LDS-DMA attention code: FSDP2 and flat-unit FSDP, same box
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 > $O/llama_fsdp2.log 2>&1 || { tail -20 $O/llama_fsdp2.log; exit 1; }
grep "{" $O/llama_fsdp2.log | tail -1 | cut -c1-400
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_flat.log 2>&1 || { tail -20 $O/llama_flat.log; exit 1; }
grep "{" $O/llama_flat.log | tail -1 | cut -c1-400
