#!/bin/bash
# parity tests, then config-4 bench lines (private + public)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --workload config4 --steps 3 --warmup 1 ${C4ARGS} > gpurun_out/c4_private.json 2> gpurun_out/c4_private.err || { echo private failed; tail -20 gpurun_out/c4_private.err; exit 1; }
cat gpurun_out/c4_private.json
timeout -k 10 300 python bench.py --workload config4 --public --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_public.json 2> gpurun_out/c4_public.err || { echo public failed; tail -20 gpurun_out/c4_public.err; exit 1; }
cat gpurun_out/c4_public.json
