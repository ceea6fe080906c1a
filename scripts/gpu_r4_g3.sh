set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_optim_overlap_gpu.py tests/test_norm_fold_gpu.py -m gpu > gpurun_out/r4/g3_norm_overlap.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_step_ab.py --steps 10 > gpurun_out/r4/g3_step_ab.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 10 --variant on > gpurun_out/r4/g3_step_nopart.log 2>&1 &&
DWAMD_NORM_FOLD_BIAS=0 timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 10 --variant on > gpurun_out/r4/g3_step_nofold.log 2>&1 &&
timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g3_bench_norm_part.log 2>&1 &&
DWAMD_NORM_BWD_PART_OFF=1 timeout -k 10 120 python -u scripts/bench_norm.py > gpurun_out/r4/g3_bench_norm_nopart.log 2>&1 &&
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_nosplit.so timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/g3_attn_nosplit.log 2>&1 &&
timeout -k 10 400 python -u bench.py --out-dir gpurun_out/r4/bench_run > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err &&
timeout -k 10 240 python -u scripts/probe_first_step.py --out gpurun_out/r4/first_step_probe.jsonl > gpurun_out/r4/g3_probe.log 2>&1 &&
timeout -k 10 200 ./scripts/probe/epi_probe wgrad > gpurun_out/r4/epi_bgrad.txt 2>&1
