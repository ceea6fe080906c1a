set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# dwamd-run --comm-perf-test on the box's GPU(s): collective sweep + link test JSON, then a short training job
timeout -k 10 300 python -u -m dlrover_wuqiong_amd.trainer.run --nnodes 1 --nproc-per-node 1 --comm-perf-test --local-addr 127.0.0.1 examples/elastic_train.py --steps 5 --ckpt-dir /tmp/r5cp > gpurun_out/r5/commperf_run.log 2>&1 &&
cp /tmp/dlrover/network_check/comm_perf_n0.json gpurun_out/r5/comm_perf_n0.json
