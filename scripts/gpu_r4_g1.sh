set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py tests/test_flash_ckpt_gpu.py -m gpu > gpurun_out/r4/g1_pytest.log 2>&1 && \
timeout -k 10 400 python -u scripts/probe_first_step.py --out gpurun_out/r4/first_step_probe.jsonl > gpurun_out/r4/g1_probe.log 2>&1
