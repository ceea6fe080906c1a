set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_rehearsal_gpu.py tests/test_optim_in_backward_gpu.py tests/test_ops_gpu.py tests/test_deterministic_gpu.py > $O/pytest.log 2>&1
echo "pytest rc $?"; tail -1 $O/pytest.log
# Llama-3-8B FSDP2: optimizer after the backward vs inside it (grid caps)
timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
for b in 0 256 64; do
  DWAMD_IN_BACKWARD_BLOCKS=$b timeout -k 10 400 python -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --optim-in-backward >> $O/fsdp.jsonl 2>> $O/fsdp.err || exit $?
  echo "blocks $b" >> $O/fsdp.jsonl
done
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --out-dir $O/run > $O/bench.json 2> $O/bench.err || exit $?
echo done
