#!/bin/bash
# Round-5 experiment 24 (r5zd): staged records per thread per write-out
# batch of the partition scatters (DPG_SCAT_WB 4, default, vs 2 and 3; the
# level-1 piece scatter spills 9 VGPRs at 4), config 2.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5zd STEPS=10 VARIANTS="cur:DPG_X=0 swb2:DPG_LIB_PATH=$L/libdpg_swb2.so swb3:DPG_LIB_PATH=$L/libdpg_swb3.so" bash tools/gpu_env_ab.sh
