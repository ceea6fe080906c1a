set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g17
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# flat-unit FSDP: GPU tests, then the Llama-3-8B step FSDP2 (zero2) vs flat (flat_zero2), then flat + flash ckpt
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flat_fsdp_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 > $O/llama_fsdp2.log 2>&1 || { tail -20 $O/llama_fsdp2.log; exit 1; }
grep "{" $O/llama_fsdp2.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_flat.log 2>&1 || { tail -20 $O/llama_flat.log; exit 1; }
grep "{" $O/llama_flat.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --steps 9 --flat --ckpt-dir /tmp/flatck > $O/llama_flat_ckpt.log 2>&1 || { tail -20 $O/llama_flat_ckpt.log; exit 1; }
grep "{" $O/llama_flat_ckpt.log
