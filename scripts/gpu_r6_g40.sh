set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g40
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# GPT2-shape attention kernels: packed QKV views vs separate tensors (serial backward)
for v in sep packed; do
F=""; [ $v = packed ] && F=--packed
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py $F 8,1024,25,25,64 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
for v in sep packed; do echo $v; python3 -c "
import csv
for r in csv.DictReader(open('$O/p_$v/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"; done
