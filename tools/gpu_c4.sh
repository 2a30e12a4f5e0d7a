#!/bin/bash
# Config-4 iteration: bench line (private selection) + phase cycles of every bounding kernel.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo bench failed; tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('ms', round(d['ms_per_step'],2), 'frac', round(d['roofline']['frac'],4), {k: v['ms'] for k, v in d['kernels'].items() if v['ms'] > 0.3})"
DPG_PHASE_TIMING=1 timeout -k 10 400 python -u bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/phase_c4.json 2> gpurun_out/phase_c4.err || { echo phase failed; tail -20 gpurun_out/phase_c4.err; exit 1; }
grep "dpg phase" gpurun_out/phase_c4.err | tail -3
