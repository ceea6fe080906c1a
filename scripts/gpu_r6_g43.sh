set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g43
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# Llama-3-8B flat step: D=128 backward LDS-DMA (in-tree) vs register staging (variant lib), alternating
A=$PWD/gpurun_ab/libdw_kernels_nodma128.so
for r in 1 2; do
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/dma$r.log 2>&1 || { tail -20 $O/dma$r.log; exit 1; }
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/nodma$r.log 2>&1 || { tail -20 $O/nodma$r.log; exit 1; }
done
for f in dma1 nodma1 dma2 nodma2; do echo $f $(grep "{" $O/$f.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['train_step_ms'], d['step_ms'])"); done
