set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g28
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# attention backward launch order A/B (dQ grid queued first), numerics with it on, two timing passes each
DWAMD_ATTN_BWD_DQ_FIRST=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -k "attn or attention" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/base$r.log 2>&1 || exit 1
DWAMD_ATTN_BWD_DQ_FIRST=1 timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/dqf$r.log 2>&1 || exit 1
done
for f in base1 dqf1 base2 dqf2; do echo $f; grep "{" $O/$f.log | cut -c1-150; done
