set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4/prof_step2
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_bgrad_gpu.py tests/test_norm_fold_gpu.py tests/test_fused_mlp_gpu.py -m gpu > gpurun_out/r4/g8_pytest.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_step_ab.py --variant off --steps 10 > gpurun_out/r4/g8_step_bgrad.log 2>&1 &&
DWAMD_WGRAD_BGRAD=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --variant off --steps 10 > gpurun_out/r4/g8_step_nobgrad.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_step_ab.py --variant off --steps 10 > gpurun_out/r4/g8_step_bgrad2.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_step2 -o run -- python3 scripts/bench_step_ab.py --variant off --steps 6 > gpurun_out/r4/prof_step2/run.log 2>&1 &&
find gpurun_out/r4/prof_step2 -name "*kernel_trace*" -delete &&
timeout -k 10 400 bash scripts/gpu_attn_pmc64.sh gpurun_out/r4/pmc64 > gpurun_out/r4/g8_pmc64.log 2>&1
