set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g41
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# (1) bias column sum on the side stream beside the dgrad / wgrad GEMMs: numerics + GPT2-1.5B step A/B
DWAMD_BGRAD_SIDE=1 timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "linear or gpt2 or Linear" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
timeout -k 10 300 python3 -u scripts/bench_step_ab.py --variant off --steps 15 >> $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
DWAMD_BGRAD_SIDE=1 timeout -k 10 300 python3 -u scripts/bench_step_ab.py --variant off --steps 15 >> $O/ab.jsonl 2> $O/ab.err || { tail $O/ab.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['env'].get('DWAMD_BGRAD_SIDE','0'), d['step_ms'], d['loss_last'])
"
# (2) packed vs separate attention kernels
bash scripts/gpu_r6_g40.sh
