#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --records 100000000 --pids 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_1e8.json 2> gpurun_out/bench_1e8.err || { echo bench1e8 failed; tail -20 gpurun_out/bench_1e8.err; exit 1; }
cat gpurun_out/bench_1e8.json
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_1e9.json 2> gpurun_out/bench_1e9.err || { echo bench1e9 failed; tail -20 gpurun_out/bench_1e9.err; exit 1; }
cat gpurun_out/bench_1e9.json
