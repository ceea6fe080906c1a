set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/prof_scratch
export HSA_ENABLE_IPC_MODE_LEGACY=0
L=gpurun_out/r5/g13_pg_late.log
AB="python -u scripts/bench_step_ab.py --steps 20 --variant off --flush-gb 8 --flush-dst shm"
timeout -k 10 200 $AB --pg nccl --pg-late >> $L 2>&1 || exit $?
timeout -k 10 200 $AB --pg nccl --pg-late --flusher-first >> $L 2>&1 || exit $?
B="--no-fault --no-frameworks --no-import-fault --out-dir"
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 300 python bench.py $B gpurun_out/r5/e_noreclaim > gpurun_out/r5/e_noreclaim.json 2> gpurun_out/r5/e_noreclaim.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/prof_scratch -o run -- python3 scripts/bench_step_ab.py --steps 2 --variant off --pg nccl > gpurun_out/r5/prof_scratch/log.txt 2>&1 || exit $?
python3 - <<'PY' > gpurun_out/r5/prof_scratch/scratch_kernels.txt
import csv, glob, collections
f = glob.glob("gpurun_out/r5/prof_scratch/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print("columns:", list(rows[0].keys()))
c = collections.Counter()
for r in rows:
    sc = r.get("Scratch_Size") or r.get("Private_Segment_Size") or "0"
    if int(sc or 0) > 0:
        c[(r["Kernel_Name"][:120], sc)] += 1
for (k, sc), n in c.most_common(50):
    print(n, sc, k)
print("kernels total", len(rows))
PY
find gpurun_out/r5/prof_scratch -name "*kernel_trace*" -delete
echo done
