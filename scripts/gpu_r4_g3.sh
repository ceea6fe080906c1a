set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_optim_overlap_gpu.py tests/test_norm_fold_gpu.py -m gpu > gpurun_out/r4/g3_norm_overlap.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 > gpurun_out/r4/g3_step_ab.log 2>&1 &&
DWAMD_NORM_FOLD_BIAS=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 10 --variant on > gpurun_out/r4/g3_step_nofold.log 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err
