set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g6
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# GPT2-1.5B training step kernel table (round 6 kernels: two-wave norm backward)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- \
  python3 scripts/bench_step_ab.py --steps 6 --variant off > $O/prof_step.log 2>&1 || exit $?
S=$(find $O/prof_step -name "*kernel_stats.csv" | head -1)
python3 scripts/summarize_prof.py $S $O/gpt2_1.5b_step_kernels.md "GPT2-1.5B training step kernels (B=8, S=1024, 1x MI355X), round 6: rocprofv3 --kernel-trace --stats of scripts/bench_step_ab.py --steps 6 --variant off (3 warm-up + 6 timed steps, model build included)" 9 || true
# norm backward alone (kernel-only times of the part + colsum kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_norm -o run -- \
  python3 scripts/bench_norm_bwd3.py > $O/prof_norm.log 2>&1 || exit $?
S=$(find $O/prof_norm -name "*kernel_stats.csv" | head -1)
python3 scripts/summarize_prof.py $S $O/norm_bwd_kernels.md "norm backward (GPT2 call, 8192 + 16384 rows, 105 calls each)" || true
find $O -name "*kernel_trace*" -delete
find $O -name "*.csv" -size +8M -delete
echo done
