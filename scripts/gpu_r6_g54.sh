set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g54
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# GPT2-1.5B step kernel table + D=64 attention PMC on the LDS-DMA attention code
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step -o run -- \
  python3 scripts/bench_step_ab.py --steps 6 --variant off > $O/prof_step.log 2>&1 || exit $?
S=$(find $O/prof_step -name "*kernel_stats.csv" | head -1)
python3 scripts/summarize_prof.py $S $O/gpt2_1.5b_step_kernels.md "GPT2-1.5B training step kernels (B=8, S=1024, 1x MI355X), round 6 final code (LDS-DMA attention staging incl. the dK/dV V image): rocprofv3 --kernel-trace --stats of scripts/bench_step_ab.py --steps 6 --variant off (3 warm-up + 6 timed steps, model build included)" 9 || true
find $O -name "*kernel_trace*" -delete
find $O -name "*.csv" -size +8M -delete
