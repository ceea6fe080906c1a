set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 10 --variant on > gpurun_out/r4/g3_step_nopart.log 2>&1 &&
timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g3_bench_norm_part.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g3_bench_norm_nopart.log 2>&1 &&
timeout -k 10 240 python -u scripts/probe_first_step.py --out gpurun_out/r4/first_step_probe.jsonl > gpurun_out/r4/g3_probe.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_flash_ckpt_gpu.py tests/test_meta_init_gpu.py tests/test_rehearsal_gpu.py -m gpu > gpurun_out/r4/g2_pytest.log 2>&1 &&
timeout -k 10 200 ./scripts/probe/epi_probe wgrad > gpurun_out/r4/epi_bgrad.txt 2>&1
