set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_optim_overlap_gpu.py -m gpu -k "norm or overlap" > gpurun_out/r4/g2_norm_overlap.log 2>&1 &&
timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g2_bench_norm_part.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g2_bench_norm_nopart.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 > gpurun_out/r4/g2_step_ab.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant on > gpurun_out/r4/g2_step_nopart.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_flash_ckpt_gpu.py tests/test_meta_init_gpu.py tests/test_rehearsal_gpu.py -m gpu > gpurun_out/r4/g2_pytest.log 2>&1
