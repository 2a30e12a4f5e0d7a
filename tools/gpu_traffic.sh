#!/bin/bash
# Calibrated HBM bytes per kernel launch (FETCH_SIZE / WRITE_SIZE passes of
# one bench step plus the calibration kernels) for the library in
# $DPG_LIB_PATH (default libdpg.so) and the workload in $BENCH_ARGS;
# results under gpurun_out/$TAG.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-traffic}
mkdir -p $O
cd /tmp
BA="--steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py $BA > $O/fetch_bench.json 2> $O/fetch.err || { echo fetch failed; tail -20 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py $BA > /dev/null 2> $O/write.err || { echo write failed; tail -20 $O/write.err; exit 1; }
if [ ! -f $R/gpurun_out/cal_fetch/run_counter_collection.csv ]; then
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/cal_fetch -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_fetch.err || { echo cal fetch failed; tail -5 $O/cal_fetch.err; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_write.err || { echo cal write failed; tail -5 $O/cal_write.err; exit 1; }
fi
cd $R
python3 tools/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv ${RECORDS:-1000000000} $O/hbm_traffic.json gpurun_out/cal_fetch/run_counter_collection.csv gpurun_out/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json | head -${LINES_OUT:-16}
