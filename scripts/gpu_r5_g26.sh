set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# 2-rank shared-GPU rehearsal hangs after the standbys publish: stacks every 60 s
DWAMD_BENCH_STACK_DUMP_S=60 timeout -k 10 420 python bench.py --gpus 2 --rehearse-shared-device --no-frameworks --timeout 300 --out-dir gpurun_out/r5/rehearsal2b > gpurun_out/r5/rehearsal2b.json 2> gpurun_out/r5/rehearsal2b.err
rc=$?; echo rehearsal_rc=$rc; exit $rc
