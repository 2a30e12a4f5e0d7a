#!/bin/bash
# per-phase cycles of the bounding kernels at config 4 (multi-wave on / off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/phase
mkdir -p $O
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo phase c4 failed; tail -20 $O/c4.err; exit 1; }
grep "dpg phase" $O/c4.err | tail -4
DPG_MW_OFF=1 DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --workload config4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4off.json 2> $O/c4off.err || { echo phase c4off failed; tail -20 $O/c4off.err; exit 1; }
grep "dpg phase" $O/c4off.err | tail -4
