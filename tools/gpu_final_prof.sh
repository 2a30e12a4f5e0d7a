#!/bin/bash
# Round evidence at HEAD, part 2: rocprofv3 kernel stats of the default bench
# (config 2) and calibrated FETCH / WRITE PMC passes of configs 2 and 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/final
mkdir -p $O
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
echo done
