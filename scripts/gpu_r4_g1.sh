set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py -m gpu -k "attn or attention" > gpurun_out/r4/attn_pytest.log 2>&1 && \
timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/attn_bench_ri1.log 2>&1 && \
DWAMD_KERNELS_LIB_AB=$GRAFT_REPO_ROOT/gpurun_ab/libdw_kernels_ri0.so timeout -k 10 150 python -u scripts/attn_bench.py > gpurun_out/r4/attn_bench_ri0.log 2>&1 && \
timeout -k 10 60 ./scripts/probe/epi_probe wgrad > gpurun_out/r4/epi_bgrad.txt 2>&1 && \
timeout -k 10 240 python -u scripts/probe_first_step.py --out gpurun_out/r4/first_step_probe.jsonl > gpurun_out/r4/g1_probe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --out-dir gpurun_out/r4/bench_run > gpurun_out/r4/bench.json 2> gpurun_out/r4/bench.err
