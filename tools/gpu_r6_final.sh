#!/bin/bash
# Round-6 evidence at HEAD in one call.  PMC traffic first, so that the bench
# lines that follow carry roofline.traffic of this very build:
#   1. GPU tests + smoke;
#   2. calibrated FETCH / WRITE passes of configs 2 and 4 -> profiles/hbm_traffic*.json
#      (read by bench.py while the library hash matches) and the calibration kernels;
#   3. rocprofv3 kernel stats of config 2;
#   4. bench lines: configs[1] (CPU baseline on), configs[3] private / public (CPU
#      baseline on), configs[4], the (N = 1e9, U = 1e6) and (N = 2e9, U = 2e7) inputs;
#   5. the config-5 host split.
# SKIP_TESTS / SKIP_PMC (steps 2-3) / SKIP_BENCH (steps 4-5) split it over calls; a
# bench-only call needs the profiles/hbm_traffic*.json of the PMC call copied back.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r6final}
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if [ -z "$SKIP_PMC" ]; then
cd /tmp
B1="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B1 > /dev/null 2> $O/pmc_fetch.err || { echo fetch failed; tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B1 > /dev/null 2> $O/pmc_write.err || { echo write failed; tail -20 $O/pmc_write.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch -o run -- $B1 --workload config4 > /dev/null 2> $O/c4_fetch.err || { echo c4 fetch failed; tail -20 $O/c4_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4_write -o run -- $B1 --workload config4 > /dev/null 2> $O/c4_write.err || { echo c4 write failed; tail -20 $O/c4_write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $R/tools/calib_fetch > $O/cal.json 2> $O/cal_fetch.err || { echo cal fetch failed; tail -5 $O/cal_fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_write.err || { echo cal write failed; tail -5 $O/cal_write.err; exit 1; }
cd $R
CAL="$O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json"
python3 tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv 1000000000 profiles/hbm_traffic.json $CAL | head -16
python3 tools/pmc_traffic.py $O/c4_fetch/run_counter_collection.csv $O/c4_write/run_counter_collection.csv 1000000000 profiles/hbm_traffic_c4.json $CAL | tail -3
cp profiles/hbm_traffic.json profiles/hbm_traffic_c4.json $O/
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err || { echo kt failed; tail -20 $O/kt.err; exit 1; }
cd $R
python3 tools/kstats.py $(find $O/kt -name "*kernel_stats.csv" | head -1) 10
fi
[ -n "$SKIP_BENCH" ] && { echo done; exit 0; }
summ() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'traffic', d['roofline'].get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; }
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench failed; tail -20 $O/bench_c2.err; exit 1; }
summ $O/bench_c2.json c2
timeout -k 10 600 python bench.py --workload config4 --steps 4 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail -20 $O/bench_c4.err; exit 1; }
summ $O/bench_c4.json c4
timeout -k 10 600 python bench.py --workload config4 --public --steps 4 --warmup 1 > $O/bench_c4p.json 2> $O/bench_c4p.err || { echo c4p failed; tail -20 $O/bench_c4p.err; exit 1; }
summ $O/bench_c4p.json c4p
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail -20 $O/bench_c5.err; exit 1; }
summ $O/bench_c5.json c5
timeout -k 10 400 python bench.py --records 1000000000 --pids 1000000 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_u1e6.json 2> $O/bench_u1e6.err || { echo u1e6 failed; tail -20 $O/bench_u1e6.err; exit 1; }
summ $O/bench_u1e6.json u1e6
timeout -k 10 400 python bench.py --records 2000000000 --pids 20000000 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_n2e9.json 2> $O/bench_n2e9.err || { echo n2e9 failed; tail -20 $O/bench_n2e9.err; exit 1; }
summ $O/bench_n2e9.json n2e9
timeout -k 10 300 python -u tools/ua_timing.py > $O/ua_timing.log 2>&1 || { echo ua_timing failed; tail -5 $O/ua_timing.log; exit 1; }
tail -2 $O/ua_timing.log
echo done
