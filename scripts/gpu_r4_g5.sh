set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4/prof_step
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# per-kernel table of the GPT2-1.5B step (overlapped update, norm fold, current kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_step -o run -- \
  python3 scripts/bench_step_ab.py --variant on --steps 6 > gpurun_out/r4/prof_step/run.log 2>&1 &&
find gpurun_out/r4/prof_step -name "*kernel_trace*" -delete
find gpurun_out/r4/prof_step -name "*.csv" -size +8M -delete
ls -R gpurun_out/r4/prof_step | head -20
