set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g37
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# in-tree: D=64 forward LDS-DMA default (64-key tiles up to S=2048); variant: D=128 dK/dV + dQ LDS-DMA
A=$PWD/gpurun_ab/libdw_kernels_dma128.so
for L in "" $A; do
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py tests/test_hf_attention.py -m gpu -k "attn or attention or varlen" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
done
for r in 1 2; do
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/base$r.log 2>&1 || exit 1
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/dma128$r.log 2>&1 || exit 1
done
for f in base1 dma1281 base2 dma1282; do echo $f; grep "{" $O/$f.log | cut -c1-150; done
for v in base dma128; do
L=""; [ $v = dma128 ] && L=$A
DWAMD_ATTN_BWD_CONCURRENT=0 DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py 4,4096,32,8,128 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
