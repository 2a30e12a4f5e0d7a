#!/bin/bash
# SQ counter passes (issue / LDS / wait breakdown per kernel) on a 2e8-record
# bench run; each pass is its own rocprofv3 run with <= 8 SQ counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
ARGS="--records ${RECORDS:-200000000} --pids ${PIDS:-2000000} --steps 1 --warmup 1 --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES" \
           "SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_IFETCH SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_INSTS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py $OUT/p*/run_counter_collection.csv > $OUT/summary.txt
cat $OUT/summary.txt
