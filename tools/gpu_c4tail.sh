#!/bin/bash
# config-4 heavy-id tail: per-step phase lines (hand-backs, big buckets)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DPG_PHASE_TIMING=1 timeout -k 10 400 python -u bench.py --workload config4 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/c4tail.json 2> gpurun_out/c4tail.err || { echo failed; tail -20 gpurun_out/c4tail.err; exit 1; }
grep "dpg phase" gpurun_out/c4tail.err | grep -v "small\|medium" | cut -c1-200
timeout -k 10 400 python -u bench.py --workload config4 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err || { echo failed; tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print('c4 ms', round(d['ms_per_step'],2), {k: round(v['ms'],2) for k, v in d['kernels'].items() if v['ms'] > 1})"
