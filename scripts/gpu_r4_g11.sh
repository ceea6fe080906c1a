set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 120 ./scripts/probe/adam_probe > gpurun_out/r4/g11_adam_probe.jsonl 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_mlp_gpu.py tests/test_ops_gpu.py -m gpu > gpurun_out/r4/g11_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 --variant off > gpurun_out/r4/g11_step.log 2>&1
