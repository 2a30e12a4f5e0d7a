#!/bin/bash
# Round-5 evidence at HEAD (both parts of tools/gpu_final.sh + gpu_final_prof.sh in one call, plus
# the timing build's phase clocks): all GPU tests + smoke, the config-2 bench
# line (with the CPU baseline), configs 4 (private, public) and 5, the
# config-5 host split; rocprofv3 kernel stats and calibrated FETCH / WRITE passes of configs 2, 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r5final}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c2.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'cpu', d.get('cpu_baseline',{}).get('value')); print({k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail -20 $O/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4 ms', round(d['ms_per_step'],2)); print({k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 400 python bench.py --workload config4 --public --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_c4p.json 2> $O/bench_c4p.err || { echo c4p failed; tail -20 $O/bench_c4p.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4p.json')); print('c4 public ms', round(d['ms_per_step'],2))"
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); print('c5 ms', round(d['ms_per_step'],2), d['stage_ms']); print(d.get('cpu_baseline'))"
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua_timing failed; tail -5 $O/ua_timing.log; exit 1; }
tail -2 $O/ua_timing.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err || { echo kt failed; tail -20 $O/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch.err || { echo fetch failed; tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/pmc_write.err || { echo write failed; tail -20 $O/pmc_write.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/c4_fetch.err || { echo c4 fetch failed; tail -20 $O/c4_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4_write -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/c4_write.err || { echo c4 write failed; tail -20 $O/c4_write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $R/tools/calib_fetch > $O/cal.json 2> $O/cal_fetch.err || { echo cal fetch failed; tail -5 $O/cal_fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_write.err || { echo cal write failed; tail -5 $O/cal_write.err; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv 1000000000 $O/hbm_traffic.json $O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json | head -16
python3 tools/pmc_traffic.py $O/c4_fetch/run_counter_collection.csv $O/c4_write/run_counter_collection.csv 1000000000 $O/hbm_traffic_c4.json $O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json | tail -3

DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/phase.json 2> $O/phase.err || { echo phase failed; tail -20 $O/phase.err; exit 1; }
grep -E "scatter phases|dpg phase" $O/phase.err | tail -3
echo done
