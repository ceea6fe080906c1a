set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g45
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# D=128 forward with 128-key tiles (variant lib): numerics, attention timing, kernel split, Llama flat step
A=$PWD/gpurun_ab/libdw_kernels_f128bk.so
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_attention_ext_gpu.py tests/test_deterministic_gpu.py tests/test_hf_attention.py -k "attn or attention or varlen" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/base$r.log 2>&1 || exit 1
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 300 python3 -u scripts/attn_bench.py > $O/bk128$r.log 2>&1 || exit 1
done
for f in base1 bk1281 base2 bk1282; do echo $f; grep "{" $O/$f.log | grep '"D": 128' | cut -c1-130; done
for v in base bk128; do
L=""; [ $v = bk128 ] && L=$A
DWAMD_KERNELS_LIB_AB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 scripts/attn_prof_run.py --fwd 4,4096,32,8,128 1,8192,32,8,128 > $O/p_$v.log 2>&1 || exit 1
done
find $O -name "*kernel_trace*" -delete
for v in base bk128; do echo $v; python3 -c "
import csv
for r in csv.DictReader(open('$O/p_$v/run_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"; done
for r in 1 2; do
timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_base$r.log 2>&1 || { tail -20 $O/llama_base$r.log; exit 1; }
DWAMD_KERNELS_LIB_AB=$A timeout -k 10 400 python3 -u scripts/bench_fsdp_llama.py --no-ckpt --steps 8 --flat > $O/llama_bk128$r.log 2>&1 || { tail -20 $O/llama_bk128$r.log; exit 1; }
done
for f in llama_base1 llama_bk1281 llama_base2 llama_bk1282; do echo $f $(grep "{" $O/$f.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['train_step_ms'])"); done
