set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g29
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u scripts/probe_llama_copies.py > $O/probe.log 2>&1 || { tail -30 $O/probe.log; exit 1; }
grep -n -i "copy\|memcpy\|contiguous\|clone\|cat" $O/probe.log | head -60
