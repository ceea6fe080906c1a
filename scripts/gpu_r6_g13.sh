set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g13
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# D=64 attention backward: baseline timing, then per-kernel standalone times (dQ not on the side stream)
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/attn_base.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/attn_serial.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $O/prof.log 2>&1 || exit 1
find $O -name "*kernel_trace*" -delete
grep "{" $O/attn_base.log; echo SERIAL; grep "{" $O/attn_serial.log
