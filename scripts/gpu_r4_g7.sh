set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4/prof_norm
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_norm_fold_gpu.py -m gpu -k "norm" > gpurun_out/r4/g7_norm_pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run3 > gpurun_out/r4/bench3.json 2> gpurun_out/r4/bench3.err &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_norm/part -o run -- python3 scripts/bench_step_ab.py --variant off --steps 4 > gpurun_out/r4/prof_norm/part.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 DWAMD_NORM_FOLD_BIAS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_norm/nopart -o run -- python3 scripts/bench_step_ab.py --variant off --steps 4 > gpurun_out/r4/prof_norm/nopart.log 2>&1 &&
find gpurun_out/r4/prof_norm -name "*kernel_trace*" -delete &&
timeout -k 10 240 python -u scripts/probe_first_step.py --out gpurun_out/r4/first_step_probe.jsonl > gpurun_out/r4/g7_probe.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_flash_ckpt_gpu.py tests/test_meta_init_gpu.py tests/test_rehearsal_gpu.py -m gpu > gpurun_out/r4/g2_pytest.log 2>&1 &&
timeout -k 10 200 ./scripts/probe/epi_probe wgrad > gpurun_out/r4/epi_bgrad.txt 2>&1
