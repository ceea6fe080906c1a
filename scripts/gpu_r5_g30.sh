set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# 2-rank shared-GPU rehearsal (no HBM tier when ranks share the card)
DWAMD_BENCH_STACK_DUMP_S=100 timeout -k 10 900 python bench.py --gpus 2 --rehearse-shared-device --no-frameworks --timeout 700 --out-dir gpurun_out/r5/rehearsal2d > gpurun_out/r5/rehearsal2d.json 2> gpurun_out/r5/rehearsal2d.err
rc=$?; echo rehearsal_rc=$rc; exit $rc
