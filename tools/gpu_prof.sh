#!/bin/bash
# rocprofv3 kernel trace + stats of the default bench, then separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) -> profiles-ready summaries in gpurun_out/prof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r1}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof/kt_bench.json 2> $R/gpurun_out/prof/kt.err || { echo kt failed; tail -20 $R/gpurun_out/prof/kt.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/pmc_fetch.err || { echo fetch failed; tail -20 $R/gpurun_out/prof/pmc_fetch.err; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/pmc_write.err || { echo write failed; tail -20 $R/gpurun_out/prof/pmc_write.err; exit 1; }
cd $R
python3 tools/pmc_traffic.py gpurun_out/prof/pmc_fetch/run_counter_collection.csv gpurun_out/prof/pmc_write/run_counter_collection.csv 1000000000 gpurun_out/prof/hbm_traffic.json
cp gpurun_out/prof/kt/run_kernel_stats.csv gpurun_out/prof/${TAG}_kernel_stats.csv
