set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py -k "replay or deferred_state" > gpurun_out/r5/g8_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -le 1 ] || exit $rc
# which part of the bench makes the steps during a checkpoint flush slower
# when the worker holds a world-1 RCCL group (b_default 150 ms vs b_nopg 108)
B="--no-fault --no-frameworks --no-import-fault --out-dir"
timeout -k 10 300 python bench.py $B gpurun_out/r5/c_default > gpurun_out/r5/c_default.json 2> gpurun_out/r5/c_default.err || exit $?
DWAMD_BENCH_PG_BACKEND=gloo timeout -k 10 300 python bench.py $B gpurun_out/r5/c_gloo > gpurun_out/r5/c_gloo.json 2> gpurun_out/r5/c_gloo.err || exit $?
DWAMD_BENCH_STANDBY=off timeout -k 10 300 python bench.py $B gpurun_out/r5/c_nosb > gpurun_out/r5/c_nosb.json 2> gpurun_out/r5/c_nosb.err || exit $?
DWAMD_STANDBY_PREFORM=0 timeout -k 10 300 python bench.py $B gpurun_out/r5/c_nopre > gpurun_out/r5/c_nopre.json 2> gpurun_out/r5/c_nopre.err || exit $?
echo done
