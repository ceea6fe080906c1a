#!/bin/bash
# PMC counters of the D=64 (GPT2-1.5B shape) attention kernels, serial backward.
set -u
OUT=${1:-gpurun_out/pmc64}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 DWAMD_ATTN_BWD_CONCURRENT=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1 -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $OUT/p2 -o run -- \
  python3 scripts/attn_prof_run.py 8,1024,25,25,64 > $OUT/p2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $OUT attn_ > $OUT/summary.txt
find $OUT -name "*kernel_trace*" -delete
echo done
