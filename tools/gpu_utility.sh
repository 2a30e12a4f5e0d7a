#!/bin/bash
# Utility-analysis GPU tests + config-5 bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |Error|error" gpurun_out/pytest_ua.log | head -30; tail -5 gpurun_out/pytest_ua.log; exit 1; }
tail -1 gpurun_out/pytest_ua.log
timeout -k 10 500 python bench.py --workload config5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo bench failed; tail -20 gpurun_out/bench_c5.err; exit 1; }
