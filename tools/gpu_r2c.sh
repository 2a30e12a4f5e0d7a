#!/bin/bash
# Round-2 re-entry HEAD check: every GPU test, smoke, config-2 / config-4 bench
# lines and a rocprofv3 kernel-stats pass of the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('c2 ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), {k: v['ms'] for k, v in d['kernels'].items() if v['ms'] > 0.3})"
timeout -k 10 400 python bench.py --workload config4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo c4 failed; tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('c4 ms', round(d['ms_per_step'],2), {k: v['ms'] for k, v in d['kernels'].items() if v['ms'] > 0.3})"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof/kt_bench.json 2> $R/gpurun_out/prof/kt.err || { echo kt failed; tail -20 $R/gpurun_out/prof/kt.err; exit 1; }
cd $R
head -12 gpurun_out/prof/kt/run_kernel_stats.csv | cut -c1-160
