#!/bin/bash
# Split k_bound_sorted's HBM fetch into value gathers and the rest: calibrated
# FETCH_SIZE / WRITE_SIZE passes of the default bench with the product
# library and with a build whose value reads return 0 (-DDPG_EXP_NO_GATHER=1,
# pipelinedp_amd/lib/libdpg_nogather.so: same records, same kept pairs, no
# gathers).  Results: gpurun_out/split/hbm_{prod,nogather}.json.
# Build the variant first, on the CPU: python tools/build_variant.py
# libdpg_nogather.so -DDPG_EXP_NO_GATHER=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
[ -f $R/pipelinedp_amd/lib/libdpg_nogather.so ] || { echo "libdpg_nogather.so missing (see header)"; exit 1; }
export TMPDIR=/tmp
O=$R/gpurun_out/split
mkdir -p $O
cd /tmp
for v in prod nogather; do
  if [ $v = nogather ]; then export DPG_LIB_PATH=$R/pipelinedp_amd/lib/libdpg_nogather.so; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${v}_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${v}_fetch.err || { echo $v fetch failed; tail -20 $O/${v}_fetch.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${v}_write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/${v}_write.err || { echo $v write failed; tail -20 $O/${v}_write.err; exit 1; }
done
unset DPG_LIB_PATH
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $R/tools/calib_fetch > $O/cal.json 2> $O/cal_fetch.err || { echo cal fetch failed; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $O/cal_write.err || { echo cal write failed; exit 1; }
cd $R
for v in prod nogather; do
  echo "== $v"
  python3 tools/pmc_traffic.py $O/${v}_fetch/run_counter_collection.csv $O/${v}_write/run_counter_collection.csv 1000000000 $O/hbm_$v.json $O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv profiles/calib/known_bytes.json > $O/summary_$v.txt; head -14 $O/summary_$v.txt
done
