set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 400 bash scripts/gpu_attn_pmc128.sh gpurun_out/r4/pmc128 > gpurun_out/r4/g4_pmc.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --model gpt2-1.5b --seq 1024 --micro-batch 8 --steps 6 --storage --ckpt-dir /tmp/dwamd_fsdp_g4 > gpurun_out/r4/g4_fsdp_gpt2_storage.json 2> gpurun_out/r4/g4_fsdp_gpt2_storage.err
