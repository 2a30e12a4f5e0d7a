#!/bin/bash
# Round-5 experiment 6: the narrow sort kernel's occupancy.  s16 = working
# set sized for 256 candidates (6 KB), 16 waves per CU as before; c128 = 128
# candidates (chunks with more go to the 2-wave kernel), 16 waves; v20 = 128
# candidates, no next-chunk prefetch, 96 VGPRs: 20 waves per CU; v20pf = v20
# with the prefetch (spills).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5h/ab VARIANTS="new:DPG_X=0 s16:DPG_LIB_PATH=$L/libdpg_s16.so c128:DPG_LIB_PATH=$L/libdpg_c128.so v20:DPG_LIB_PATH=$L/libdpg_v20.so v20pf:DPG_LIB_PATH=$L/libdpg_v20pf.so" bash tools/gpu_env_ab.sh
