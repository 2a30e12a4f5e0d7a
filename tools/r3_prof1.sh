# round-3: where the small-chunk bounding kernel spends its time (phase cycles
# of both small-chunk kernels, SQ issue/wait split at 2e8 records)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r3p
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r3p/phase_sort.json 2> gpurun_out/r3p/phase_sort.err || { echo phase failed; tail -20 gpurun_out/r3p/phase_sort.err; exit 1; }
grep "dpg phase" gpurun_out/r3p/phase_sort.err | tail -2
DPG_BOUND_HASH=1 DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r3p/phase_hash.json 2> gpurun_out/r3p/phase_hash.err || { echo phase hash failed; tail -20 gpurun_out/r3p/phase_hash.err; exit 1; }
grep "dpg phase" gpurun_out/r3p/phase_hash.err | tail -2
cd /tmp
ARGS="--records 200000000 --pids 2000000 --steps 1 --warmup 1 --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  for kern in sort hash; do
    E=""
    [ $kern = hash ] && E="DPG_BOUND_HASH=1"
    export DPG_BOUND_HASH_SET=$kern
    if [ $kern = hash ]; then export DPG_BOUND_HASH=1; else unset DPG_BOUND_HASH; fi
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/r3p/p${i}_$kern -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/r3p/p${i}_$kern.log 2>&1 || { echo "pass $i $kern failed"; tail -5 $R/gpurun_out/r3p/p${i}_$kern.log; exit 1; }
  done
done
unset DPG_BOUND_HASH
cd $R
for kern in sort hash; do
  echo "== $kern"
  python3 tools/pmc_summary.py gpurun_out/r3p/p*_$kern/run_counter_collection.csv > gpurun_out/r3p/summary_$kern.txt
  grep -A 40 "k_bound" gpurun_out/r3p/summary_$kern.txt | head -45
done
