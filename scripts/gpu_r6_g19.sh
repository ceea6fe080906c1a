set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g19
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# module_replace now swaps nn.Linear -> FusedLinear: flat FSDP + FSDP2 Llama-3-8B steps, flat kernel table
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flat_fsdp_gpu.py tests/test_amp_gpu.py tests/test_fp8_gpu.py tests/test_meta_init_gpu.py tests/test_optim_in_backward_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_flat.log 2>&1 || { tail -20 $O/llama_flat.log; exit 1; }
grep "{" $O/llama_flat.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 > $O/llama_fsdp2.log 2>&1 || { tail -20 $O/llama_fsdp2.log; exit 1; }
grep "{" $O/llama_fsdp2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O -name "*kernel_trace*" -delete
