set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g30
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# Llama-3-8B flat FSDP built on the meta device (each rank fills its shard) vs built full, then flat GPU tests
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flat_fsdp_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat --meta > $O/meta.log 2>&1 || { tail -20 $O/meta.log; exit 1; }
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 4 --flat > $O/full.log 2>&1 || { tail -20 $O/full.log; exit 1; }
grep "{" $O/meta.log | cut -c1-520; grep "{" $O/full.log | cut -c1-520
