set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g18
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# flat-unit FSDP Llama-3-8B: flash-ckpt run, then the step's kernel table
timeout -k 10 500 python3 -u scripts/bench_fsdp_llama.py --steps 9 --flat --ckpt-dir /tmp/flatck > $O/llama_flat_ckpt.log 2>&1 || { tail -20 $O/llama_flat_ckpt.log; exit 1; }
grep "{" $O/llama_flat_ckpt.log
rm -rf /tmp/flatck
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O -name "*kernel_trace*" -delete
grep "{" $O/prof.log
