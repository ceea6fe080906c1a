set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g52
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# dK/dV kernel: the block's V image by LDS-DMA (variant lib): numerics + kernel split at the GPT2 and Llama shapes
A=$PWD/gpurun_ab/libdw_kernels_vdma.so
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py tests/test_hf_attention.py -k "attn or attention or varlen" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for v in base vdma; do
L=""; [ $v = vdma ] && L=$A
DWAMD_ATTN_BWD_CONCURRENT=0 DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v$r -o run -- python3 scripts/attn_prof_run.py --packed 8,1024,25,25,64 > $O/p_$v$r.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q_$v$r -o run -- python3 scripts/attn_prof_run.py 1,4096,32,8,128 > $O/q_$v$r.log 2>&1 || exit 1
done
done
find $O -name "*kernel_trace*" -delete
for v in p_base1 p_vdma1 p_base2 p_vdma2 q_base1 q_vdma1 q_base2 q_vdma2; do echo $v; python3 -c "
import csv
for r in csv.DictReader(open('$O/$v/run_kernel_stats.csv')):
    if 'dkdv' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'])
"; done
