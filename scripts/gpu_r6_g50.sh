set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g50
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# Llama-3-8B flat-FSDP step kernel table on the round's final kernels (LDS-DMA attention, quad norm backward)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O -name "*kernel_trace*" -delete
grep "{" $O/prof.log | cut -c1-400
S=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/summarize_prof.py $S $O/llama3_8b_flat_fsdp_kernels.md "Llama-3-8B flat-unit FSDP step (flat_zero2, bf16 params + fp32 masters in FusedAdamW, S=4096, 1x MI355X), round 6 final kernels (LDS-DMA attention staging, wave-quad norm backward): rocprofv3 --kernel-trace --stats of scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat (2 warm-up + 4 timed steps, model build included)" 6 || true
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_flat.log 2>&1 || { tail -20 $O/llama_flat.log; exit 1; }
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 > $O/llama_fsdp2.log 2>&1 || { tail -20 $O/llama_fsdp2.log; exit 1; }
for f in llama_flat llama_fsdp2; do echo $f $(grep "{" $O/$f.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['train_step_ms'], d['tokens_per_s'])"); done
