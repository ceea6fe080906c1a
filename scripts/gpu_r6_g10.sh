set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g10
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_flash_ckpt_gpu.py tests/test_hbm_tier_gpu.py > $O/pytest.log 2>&1
echo "pytest rc $?"; tail -1 $O/pytest.log
DWAMD_CKPT_SLOTS=1 timeout -k 10 500 python -u scripts/bench_tp_shard_ring.py --staging ring --ring-hbm-gb 64 --ckpt-dir /tmp/r6ring > $O/tp8_ring64_defer.json 2> $O/tp8_ring64_defer.err || exit $?
echo done
