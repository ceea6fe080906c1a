set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# 1) norm backward (GPT2 call: LayerNorm H=1600, dres + dsum): in-tree vs two waves per SIMD, alternating
for i in 1 2; do
  timeout -k 10 120 python -u scripts/bench_norm_bwd3.py >> $O/norm.jsonl 2>> $O/norm.err || exit $?
  DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_w2.so timeout -k 10 120 python -u scripts/bench_norm_bwd3.py >> $O/norm.jsonl 2>> $O/norm.err || exit $?
done
# 2) GPT2-1.5B step, in-tree vs w2
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off >> $O/step.jsonl 2>> $O/step.err || exit $?
DWAMD_KERNELS_LIB_AB=$PWD/gpurun_ab/libdw_kernels_w2.so timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off >> $O/step.jsonl 2>> $O/step.err || exit $?
# 3) Llama-3-8B FSDP2 step: optimizer after the backward vs inside it
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --optim-in-backward >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
# 4) the fixed replay test + the import-mode allocation counter in the bench
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_flash_ckpt_gpu.py -k "replay or ring" > $O/pytest.log 2>&1
echo "pytest rc $?"
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --no-frameworks --out-dir $O/run > $O/bench.json 2> $O/bench.err || exit $?
echo done
