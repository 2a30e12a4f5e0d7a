#!/bin/bash
# Round evidence at HEAD: all GPU tests, smoke, the default bench line (with
# the CPU baseline), config-4 line, rocprofv3 kernel stats, FETCH/WRITE PMC
# passes of the default bench and of the calibration kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), 'cpu', d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo c4 failed; tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('c4 ms', round(d['ms_per_step'],2))"
timeout -k 10 400 python bench.py --workload config4 --public --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4p.json 2> gpurun_out/bench_c4p.err || { echo c4p failed; tail -20 gpurun_out/bench_c4p.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4p.json')); print('c4 public ms', round(d['ms_per_step'],2))"
timeout -k 10 400 python bench.py --workload config5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo c5 failed; tail -20 gpurun_out/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c5.json')); print('c5 ms', round(d['ms_per_step'],2))"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof/kt_bench.json 2> $R/gpurun_out/prof/kt.err || { echo kt failed; tail -20 $R/gpurun_out/prof/kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/pmc_fetch.err || { echo fetch failed; tail -20 $R/gpurun_out/prof/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/pmc_write.err || { echo write failed; tail -20 $R/gpurun_out/prof/pmc_write.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/c4_fetch -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/c4_fetch.err || { echo c4 fetch failed; tail -20 $R/gpurun_out/prof/c4_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/c4_write -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/prof/c4_write.err || { echo c4 write failed; tail -20 $R/gpurun_out/prof/c4_write.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/cal_fetch -o run -- $R/tools/calib_fetch > $R/gpurun_out/prof/cal.json 2> $R/gpurun_out/prof/cal_fetch.err || { echo cal fetch failed; tail -5 $R/gpurun_out/prof/cal_fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/cal_write -o run -- $R/tools/calib_fetch > /dev/null 2> $R/gpurun_out/prof/cal_write.err || { echo cal write failed; tail -5 $R/gpurun_out/prof/cal_write.err; exit 1; }
cd $R
echo done
