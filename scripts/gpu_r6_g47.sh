set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g47
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# norm backward for 2048 <= H <= 4096 on wave quads (variant lib): numerics, Llama call timing, Llama flat step
A=$PWD/gpurun_ab/libdw_kernels_quad.so
for L in "" $A; do
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_deterministic_gpu.py tests/test_norm_fold_gpu.py tests/test_llama.py -k "norm or llama or Norm" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
done
for r in 1 2; do
timeout -k 10 120 python3 -u scripts/bench_norm_bwd3.py --llama > $O/nb_base$r.log 2>&1 || { tail $O/nb_base$r.log; exit 1; }
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 120 python3 -u scripts/bench_norm_bwd3.py --llama > $O/nb_quad$r.log 2>&1 || { tail $O/nb_quad$r.log; exit 1; }
done
cat $O/nb_base1.log $O/nb_quad1.log $O/nb_base2.log $O/nb_quad2.log
for r in 1 2; do
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_base$r.log 2>&1 || { tail -20 $O/llama_base$r.log; exit 1; }
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_quad$r.log 2>&1 || { tail -20 $O/llama_quad$r.log; exit 1; }
done
for f in llama_base1 llama_quad1 llama_base2 llama_quad2; do echo $f $(grep "{" $O/$f.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['train_step_ms'])"); done
