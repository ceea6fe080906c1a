set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g26
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# norm backward kernel split (pair kernel vs one-wave kernel, + the column-sum pass)
for v in 0 1; do
DWAMD_NORM_BWD_PAIR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python3 scripts/bench_norm_bwd3.py > $O/p$v.log 2>&1 || { tail $O/p$v.log; exit 1; }
done
find $O -name "*kernel_trace*" -delete
for v in 0 1; do echo PAIR=$v; grep -h "norm_bwd\|colsum" $O/p$v/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-140; done
