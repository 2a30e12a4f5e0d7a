#!/bin/bash
# Round-5 experiment 5: one 64-bit atomic reserving both of a thread's runs
# in the level-1 scatter (issued before / after the scan's barrier).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5g/ab VARIANTS="new:DPG_X=0 pair:DPG_LIB_PATH=$L/libdpg_pair.so pairlate:DPG_LIB_PATH=$L/libdpg_pairlate.so" bash tools/gpu_env_ab.sh
