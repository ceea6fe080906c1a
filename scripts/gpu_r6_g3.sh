set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# whole GPU suite + smoke, as the driver runs them at round end
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
echo "pytest rc $?"; tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
# Llama-3-8B FSDP2 step with the optimizer inside the backward: kernel trace -> overlap of the update
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ib -o run -- \
  python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --optim-in-backward > $O/prof_ib.log 2>&1 || exit $?
T=$(find $O/prof_ib -name "*kernel_trace.csv" | head -1)
S=$(find $O/prof_ib -name "*kernel_stats.csv" | head -1)
python3 scripts/overlap_stats.py $T mt_step_kernel > $O/overlap_ib.json
python3 scripts/summarize_prof.py $S $O/llama3_8b_fsdp_in_backward_kernels.md "Llama-3-8B FSDP2 step, optimizer inside the backward" 6 || true
find $O/prof_ib -name "*kernel_trace*" -delete
find $O/prof_ib -name "*.csv" -size +8M -delete
# Llama-3 70B TP=8 shard on a forced 64 GB ring: the deferred write-back's plan vs the run's HBM peak
DWAMD_CKPT_SLOTS=1 timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging ring --ring-hbm-gb 64 --ckpt-dir /tmp/r6ring > $O/tp8_ring64_defer.json 2> $O/tp8_ring64_defer.err || exit $?
echo done
