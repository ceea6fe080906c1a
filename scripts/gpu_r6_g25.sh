set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g25
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
# norm backward with two waves per row (H 1025..2047): numerics, kernel alone on/off, GPT2 step on/off
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_norm_fold_gpu.py tests/test_deterministic_gpu.py -k "norm" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DWAMD_NORM_BWD_PAIR=0 timeout -k 10 200 python3 -u scripts/bench_norm_bwd3.py > $O/norm_off.log 2>&1 || { tail $O/norm_off.log; exit 1; }
timeout -k 10 200 python3 -u scripts/bench_norm_bwd3.py > $O/norm_on.log 2>&1 || { tail $O/norm_on.log; exit 1; }
echo OFF; grep "{" $O/norm_off.log; echo ON; grep "{" $O/norm_on.log
timeout -k 10 400 python3 -u scripts/bench_step_ab.py --steps 10 --variant off --env DWAMD_NORM_BWD_PAIR=0 > $O/step_off.log 2>&1 || { tail $O/step_off.log; exit 1; }
timeout -k 10 400 python3 -u scripts/bench_step_ab.py --steps 10 --variant off > $O/step_on.log 2>&1 || { tail $O/step_on.log; exit 1; }
echo STEP_OFF; grep "{" $O/step_off.log | tail -2; echo STEP_ON; grep "{" $O/step_on.log | tail -2
