#!/bin/bash
# Round-5 experiment 20: where the 5-wave narrow sort kernel keeps its bound
# parameters (DPG_SORT_VREG: 0 = scalar registers, 1 = the 64-bit ones in
# vector registers (default), 2 = all of them), config 2.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5z/ab STEPS=10 VARIANTS="cur:DPG_X=0 vreg0:DPG_LIB_PATH=$L/libdpg_vreg0.so vreg2:DPG_LIB_PATH=$L/libdpg_vreg2.so" bash tools/gpu_env_ab.sh
