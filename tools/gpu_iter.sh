#!/bin/bash
# One build->measure iteration on the GPU box: parity tests, phase timing,
# the 1e9 bench.  Every GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit 1; }
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo phase failed; tail -20 gpurun_out/phase.err; exit 1; }
grep "dpg phase" gpurun_out/phase.err | tail -2
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac']); print(d['stage_ms']); print(d.get('cpu_baseline'))"
