#!/bin/bash
# Diagnostics of the config-2 path in one call: the phase clock of the
# timing build (libdpg_timing.so), a rocprofv3 kernel trace with stats, and
# SQ counter passes (issue / wait / LDS / VMEM breakdown per kernel), each
# pass its own rocprofv3 run.  $TAG names gpurun_out/$TAG/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
T=${TAG:-diag}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
ARGS="--records ${RECORDS:-1000000000} --pids ${PIDS:-10000000} --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
cd $R
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py $ARGS > $OUT/phase.json 2> $OUT/phase.err || { echo phase failed; tail -20 $OUT/phase.err; exit 1; }
grep "dpg" $OUT/phase.err | tail -6
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/bench.py ${ARGS/--steps 1/--steps 3} > $OUT/kt.log 2>&1 || { echo kt failed; tail -5 $OUT/kt.log; exit 1; }
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INSTS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 tools/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) > $OUT/kstats.txt 2>&1 || true
python3 tools/pmc_summary.py $(find $OUT -path "*p[0-9]*" -name "*counter_collection.csv") > $OUT/summary.txt
cat $OUT/kstats.txt | head -12
cat $OUT/summary.txt | head -80
