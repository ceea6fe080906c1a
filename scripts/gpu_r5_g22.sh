set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# the multi-rank fault path rehearsed: 2 ranks sharing this GPU over gloo
# (4 full GPT2-1.5B replicas + 4 deep standbys do not fit one 288 GB card)
timeout -k 10 1000 python bench.py --gpus 2 --rehearse-shared-device --no-frameworks --out-dir gpurun_out/r5/rehearsal2 > gpurun_out/r5/rehearsal2.json 2> gpurun_out/r5/rehearsal2.err
rc=$?; echo rehearsal_rc=$rc; exit $rc
