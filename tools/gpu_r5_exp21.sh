#!/bin/bash
# r5za: config 5's pre-aggregate with 8-byte records and a value gather by
# record index (DPG_PA_GATHER=1), which lets the histogram-free level 1 and
# the team level 2 run (both take 8-byte records only), against the 16-byte
# records that carry the value through both levels (default).
set -o pipefail
export TMPDIR=/tmp
TAG=r5za VARIANTS="r16:DPG_X=0 gather:DPG_PA_GATHER=1" BENCH_ARGS="--workload config5" STEPS=3 \
  bash tools/gpu_env_ab.sh
