set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/g12
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
# PMC of the norm backward (GPT2 call) -- where do its 35 us go?
P1="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o run -- python3 scripts/bench_norm_bwd3.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- python3 scripts/bench_norm_bwd3.py > $O/p2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O norm_bwd_part > $O/summary.txt
python3 scripts/pmc_summary.py $O colsum >> $O/summary.txt
find $O -name "*kernel_trace*" -delete
echo done
