set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/prof_fsdp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 6 > gpurun_out/r5/fsdp_amp.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 6 --precision half > gpurun_out/r5/fsdp_half.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_fsdp -o run -- python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 > gpurun_out/r5/prof_fsdp/bench.log 2>&1 &&
find gpurun_out/r5/prof_fsdp -name "*kernel_trace*" -delete &&
find gpurun_out/r5/prof_fsdp -name "*.csv" -size +8M -delete
