#!/bin/bash
# Round-5 experiment 23 (r5zc): staged records per thread per write-out
# batch of the team level 2 (DPG_TEAM_WB 4, default, vs 8 and 2), config 2.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5zc STEPS=10 VARIANTS="cur:DPG_X=0 twb8:DPG_LIB_PATH=$L/libdpg_twb8.so twb2:DPG_LIB_PATH=$L/libdpg_twb2.so" bash tools/gpu_env_ab.sh
