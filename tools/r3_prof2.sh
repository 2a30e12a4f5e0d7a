# round-3: phase cycles + SQ issue/wait split of the narrow sort kernel
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r3q
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r3q/phase_sort.json 2> gpurun_out/r3q/phase_sort.err || { echo phase failed; tail -20 gpurun_out/r3q/phase_sort.err; exit 1; }
grep "dpg phase" gpurun_out/r3q/phase_sort.err | tail -1
cd /tmp
ARGS="--records 200000000 --pids 2000000 --steps 1 --warmup 1 --no-cpu-baseline"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/r3q/p${i} -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/r3q/p${i}.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/r3q/p${i}.log; exit 1; }
done
cd $R
python3 tools/pmc_summary.py gpurun_out/r3q/p*/run_counter_collection.csv > gpurun_out/r3q/summary.txt
grep -A 32 "k_bound_sorted" gpurun_out/r3q/summary.txt | head -70
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3q/c2.json 2> gpurun_out/r3q/c2.err || { echo bench failed; tail -20 gpurun_out/r3q/c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3q/c2.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4)); print({k: v['ms'] for k, v in d['kernels'].items()})"
