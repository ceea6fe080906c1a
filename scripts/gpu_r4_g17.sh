set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4/prof_step17
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# per-kernel table of the GPT2-1.5B step as bench.py runs it (lazy zero, default kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_step17 -o run -- \
  python3 scripts/bench_step_ab.py --variant off --steps 6 > gpurun_out/r4/prof_step17/run.log 2>&1 &&
find gpurun_out/r4/prof_step17 -name "*kernel_trace*" -delete
find gpurun_out/r4/prof_step17 -name "*.csv" -size +8M -delete
ls -R gpurun_out/r4/prof_step17 | head -20
