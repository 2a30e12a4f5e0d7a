#!/bin/bash
# Round-5 experiment 4: the piece-mode level-1 scatter's phase clock, and
# what its stores cost (a no-store diagnostic build, wrong results).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/phase.json 2> $O/phase.err || { echo phase failed; tail -20 $O/phase.err; exit 1; }
grep "scatter phases" $O/phase.err | tail -2
L=pipelinedp_amd/lib
TAG=r5f/ab VARIANTS="new:DPG_X=0 nostore:DPG_LIB_PATH=$L/libdpg_nostore.so" bash tools/gpu_env_ab.sh
