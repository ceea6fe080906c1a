set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export HSA_ENABLE_IPC_MODE_LEGACY=0
# norm backward (H < 2048): PF register sets per wave (rows in flight), A/B against the default 2
P3=$PWD/gpurun_ab/libdw_kernels_pf3.so
P4=$PWD/gpurun_ab/libdw_kernels_pf4.so
DWAMD_KERNELS_LIB_AB=$P4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_fused_mlp_gpu.py -k "norm or layer or gpt2" > gpurun_out/r5/pf_pytest.log 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$P3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "norm or layer" >> gpurun_out/r5/pf_pytest.log 2>&1 || exit $?
for v in base $P3 $P4 base $P3 $P4; do
  if [ "$v" = base ]; then
    echo "{\"variant\": \"base\"}" >> gpurun_out/r5/pf_step.log
    timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off >> gpurun_out/r5/pf_step.log 2>&1 || exit $?
  else
    echo "{\"variant\": \"$(basename $v)\"}" >> gpurun_out/r5/pf_step.log
    DWAMD_KERNELS_LIB_AB=$v timeout -k 10 200 python -u scripts/bench_step_ab.py --steps 20 --variant off >> gpurun_out/r5/pf_step.log 2>&1 || exit $?
  fi
done
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/prof_pf_base gpurun_out/r5/prof_pf4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_pf_base -o run -- python3 scripts/bench_step_ab.py --steps 6 --variant off > gpurun_out/r5/prof_pf_base/log.txt 2>&1 || exit $?
DWAMD_KERNELS_LIB_AB=$P4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_pf4 -o run -- python3 scripts/bench_step_ab.py --steps 6 --variant off > gpurun_out/r5/prof_pf4/log.txt 2>&1 || exit $?
echo done
