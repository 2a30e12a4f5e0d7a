#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the config-4 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/c4prof
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/c4prof/fetch -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/c4prof/fetch.err || { echo fetch failed; tail -20 $R/gpurun_out/c4prof/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/c4prof/write -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/c4prof/write.err || { echo write failed; tail -20 $R/gpurun_out/c4prof/write.err; exit 1; }
cd $R
python3 tools/pmc_traffic.py gpurun_out/c4prof/fetch/run_counter_collection.csv gpurun_out/c4prof/write/run_counter_collection.csv 1000000000 gpurun_out/c4prof/hbm_traffic_c4.json
