set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g15
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# wide D=64 dK/dV kernel (DWAMD_ATTN_DKDV64W=1): numerics, then timing against the 3-wave kernel
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py -k "attn or attention" > $O/pytest_base.log 2>&1 || { tail -30 $O/pytest_base.log; exit 1; }
DWAMD_ATTN_DKDV64W=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py -k "attn or attention" > $O/pytest_w.log 2>&1 || { tail -30 $O/pytest_w.log; exit 1; }
tail -2 $O/pytest_w.log
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/attn_base.log 2>&1 || exit 1
DWAMD_ATTN_DKDV64W=1 timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/attn_w.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 DWAMD_ATTN_DKDV64W=1 timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/attn_w_serial.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_base -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $O/prof_base.log 2>&1 || exit 1
DWAMD_ATTN_BWD_CONCURRENT=0 DWAMD_ATTN_DKDV64W=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $O/prof_w.log 2>&1 || exit 1
find $O -name "*kernel_trace*" -delete
echo BASE; grep "{" $O/attn_base.log; echo WIDE; grep "{" $O/attn_w.log; echo WIDE_SERIAL; grep "{" $O/attn_w_serial.log
for d in prof_base prof_w; do echo $d; grep -h "attn_bwd" $O/$d/*kernel_stats.csv | cut -c1-160; done
