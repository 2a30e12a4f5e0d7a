#!/bin/bash
# Round-5 closing evidence at the final library: tools/gpu_r5_final.sh
# (GPU suite, smoke, bench lines, host split, rocprofv3 kernel stats, PMC
# traffic, phase clocks), then a same-box config-2 A/B of the partition
# scatters' 2-record write-out batch (DPG_SCAT_WB=2) against the previous
# build (libdpg_prev.so).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${TAG:-r5final7} bash tools/gpu_r5_final.sh || exit 1
TAG=${TAG:-r5final7}/ab STEPS=10 VARIANTS="new:DPG_X=0 prev:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_prev.so" bash tools/gpu_env_ab.sh
