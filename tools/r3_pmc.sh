#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the default bench (config 2) and of the
# calibration kernels -> calibrated HBM bytes per kernel launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/fetch_bench.json 2> $O/fetch.err || { echo fetch failed; tail -20 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/write.err || { echo write failed; tail -20 $O/write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $R/tools/calib_fetch > $O/cal.json 2> $O/cal_fetch.err || { echo cal fetch failed; tail -5 $O/cal_fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_write.err || { echo cal write failed; tail -5 $O/cal_write.err; exit 1; }
cd $R
python3 tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv 1000000000 $O/hbm_traffic.json $O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json
