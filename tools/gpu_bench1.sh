#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --records 100000000 --pids 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1e8.json 2> gpurun_out/bench_1e8.err || { echo bench1e8 failed; tail -20 gpurun_out/bench_1e8.err; exit 1; }
cat gpurun_out/bench_1e8.json
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_1e9.json 2> gpurun_out/bench_1e9.err || { echo bench1e9 failed; tail -20 gpurun_out/bench_1e9.err; exit 1; }
cat gpurun_out/bench_1e9.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || { echo rocprof failed; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof1.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
