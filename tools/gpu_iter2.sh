#!/bin/bash
# Kernel iteration: parity tests of the bounding kernels, default bench line, phase cycles.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { echo pytest failed; grep -E "^E |Error|FAILED" gpurun_out/pytest_iter.log | head -20; tail -3 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { echo bench failed; tail -20 gpurun_out/bench_iter.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_iter.json')); print('ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), {k: v['ms'] for k, v in d['kernels'].items() if v['ms'] > 0.3})"
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo phase failed; tail -20 gpurun_out/phase.err; exit 1; }
grep "dpg phase" gpurun_out/phase.err | tail -1
