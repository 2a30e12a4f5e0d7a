#!/bin/bash
# Round-5 experiment 22 (r5zb): items per thread of the utility
# pre-aggregate's item levels at config 5: 24-byte pairs (items and pairs
# levels) 4 (default) -> 5 (the LDS stage caps it there; the 16-byte record
# levels are at their LDS cap already).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5zb STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="cur:DPG_X=0 iw5:DPG_LIB_PATH=$L/libdpg_iw5.so" bash tools/gpu_env_ab.sh
