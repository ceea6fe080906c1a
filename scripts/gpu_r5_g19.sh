set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/prof_step
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# fresh GPT2-1.5B step kernel table (round-5 kernels)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_step -o run -- python3 scripts/bench_step_ab.py --steps 6 --variant off > gpurun_out/r5/prof_step/log.txt 2>&1 || exit $?
find gpurun_out/r5/prof_step -name "*kernel_trace*" -delete
# the multi-rank fault path rehearsed: 4 ranks sharing this GPU over gloo (sliced saves, SIGKILL, restarts)
timeout -k 10 900 python bench.py --gpus 4 --rehearse-shared-device --no-frameworks --out-dir gpurun_out/r5/rehearsal4 > gpurun_out/r5/rehearsal4.json 2> gpurun_out/r5/rehearsal4.err
rc=$?; echo rehearsal_rc=$rc; exit $rc
