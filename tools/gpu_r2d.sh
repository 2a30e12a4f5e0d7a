#!/bin/bash
# histogram + utility GPU tests, then default bench with phase cycles
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_histograms.py tests/test_gpu_utility.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo phase failed; tail -20 gpurun_out/phase.err; exit 1; }
grep "dpg phase" gpurun_out/phase.err | tail -2
