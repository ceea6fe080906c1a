set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g51
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# D=64 forward at S=2048: 64-key tiles (in-tree, up to S=2048) vs 128-key tiles (variant: threshold 1024)
A=$PWD/gpurun_ab/libdw_kernels_thr1k.so
for v in base thr1k; do
L=""; [ $v = thr1k ] && L=$A
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py --fwd 4,2048,25,25,64 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
for v in base thr1k; do echo $v; python3 -c "
import csv
for r in csv.DictReader(open('$O/p_$v/run_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
"; done
