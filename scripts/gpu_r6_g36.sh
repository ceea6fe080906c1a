set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g36
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# D=64 forward K/V staging by LDS-DMA (variant libs: 128-key tiles, 64-key tiles): numerics, timing, kernel split
A=$PWD/gpurun_ab/libdw_kernels_fdma.so
B=$PWD/gpurun_ab/libdw_kernels_fdma64.so
for L in $A $B; do
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py -k "attn or attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
done
for r in 1 2; do
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/base$r.log 2>&1 || exit 1
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/fdma$r.log 2>&1 || exit 1
DWAMD_KERNELS_LIB_AB=$B timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/fdma64$r.log 2>&1 || exit 1
done
for f in base1 fdma1 fdma641 base2 fdma2 fdma642; do echo $f; grep "{" $O/$f.log | grep '"D": 64' | cut -c1-130; done
for v in base fdma fdma64; do
L=""; [ $v = fdma ] && L=$A; [ $v = fdma64 ] && L=$B
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py --fwd 8,1024,25,25,64 2,4096,16,16,64 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
for v in base fdma fdma64; do echo $v; grep -h "attn_fwd" $O/p_$v/*kernel_stats.csv | cut -d, -f1-6 | cut -c1-40,150-260; done
