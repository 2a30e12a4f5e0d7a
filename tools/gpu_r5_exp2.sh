#!/bin/bash
# Round-5 experiment 2: scatter phase clocks after the LDS digit bases, and
# a same-box A/B of the product library vs the round-4 base, the no-lbase
# build and the histogram-free level 1 (pieces) with the team prefetch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/phase.json 2> $O/phase.err || { echo phase failed; tail -20 $O/phase.err; exit 1; }
grep "scatter phases" $O/phase.err | tail -2
L=pipelinedp_amd/lib
TAG=r5d/ab VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=$L/libdpg_base.so nolb:DPG_LIB_PATH=$L/libdpg_nolb.so pieces:DPG_L1_PIECES=1 basepieces:DPG_LIB_PATH=$L/libdpg_base.so,DPG_L1_PIECES=1" bash tools/gpu_env_ab.sh
