set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_ckpt_gpu.py tests/test_deterministic_gpu.py tests/test_optim_overlap_gpu.py tests/test_ops_gpu.py > gpurun_out/r5/g2_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc
# test failures (1) are read afterwards; anything else (fault, abort, timeout) ends the GPU work here
[ $rc -le 1 ] || exit $rc
B="--no-fault --no-frameworks --out-dir"
timeout -k 10 300 python bench.py $B gpurun_out/r5/b_default > gpurun_out/r5/b_default.json 2> gpurun_out/r5/b_default.err &&
DWAMD_BENCH_PG_WORLD1=0 timeout -k 10 300 python bench.py $B gpurun_out/r5/b_nopg > gpurun_out/r5/b_nopg.json 2> gpurun_out/r5/b_nopg.err &&
DWAMD_FLUSH_STREAM=cumask timeout -k 10 300 python bench.py $B gpurun_out/r5/b_cumask > gpurun_out/r5/b_cumask.json 2> gpurun_out/r5/b_cumask.err &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r5/g2_step_default.log 2>&1 &&
DWAMD_DETERMINISTIC=1 timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 20 --variant off > gpurun_out/r5/g2_step_det.log 2>&1
