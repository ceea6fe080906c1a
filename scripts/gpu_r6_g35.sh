set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g35
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# D=64 dQ kernel K/V staging by LDS-DMA (variant lib): numerics, then timing vs the in-tree kernel, kernel split
L=$PWD/gpurun_ab/libdw_kernels_dqdma.so
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py -k "attn or attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/base$r.log 2>&1 || exit 1
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/dma$r.log 2>&1 || exit 1
done
for f in base1 dma1 base2 dma2; do echo $f; grep "{" $O/$f.log | head -2 | cut -c1-150; done
for v in base dma; do
if [ $v = dma ]; then export DWAMD_KERNELS_LIB_AB=$L; fi
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
for v in base dma; do echo $v; grep -h "attn_bwd_dq" $O/p_$v/*kernel_stats.csv | cut -d, -f1-6 | cut -c1-40,150-260; done
