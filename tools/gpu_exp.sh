#!/bin/bash
# Level-split experiment: partition kernel times for b1 = 11 / 10 / 9.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/exp_$name.json 2> gpurun_out/exp_$name.err || { echo "$name failed"; tail -5 gpurun_out/exp_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/exp_$name.json')); print('$name', 'ms', round(d['ms_per_step'],2), {k: round(v['ms'],2) for k, v in d['kernels'].items() if v['ms'] > 0.3})"
}
run b11 DPG_X=0
run b10 DPG_DEBUG_TARGET=512
run b9 DPG_DEBUG_TARGET=1024 DPG_DEBUG_B1=9
run b8 DPG_DEBUG_TARGET=2048 DPG_DEBUG_B1=8
