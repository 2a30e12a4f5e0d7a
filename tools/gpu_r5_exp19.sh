#!/bin/bash
# Round-5 experiment 19: the narrow sort kernel at 5 waves per SIMD with its
# full 256-candidate capacity (working set sized for 256 candidates, 96
# VGPRs: no next-chunk prefetch, 7 spilled VGPRs) against the same code at 4
# waves per SIMD with the prefetch (w4); both built from the round-5
# three-tier sources with the mid tier off.  Compare the bounding stages.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
DPG_LIB_PATH=$L/libdpg_w5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "bounding_triggered or level2_paths and pieces" > gpurun_out/r5w_pytest.log 2>&1 || { echo pytest failed; tail -20 gpurun_out/r5w_pytest.log; exit 1; }
tail -1 gpurun_out/r5w_pytest.log
TAG=r5w/ab STEPS=10 VARIANTS="cur:DPG_X=0 w4:DPG_LIB_PATH=$L/libdpg_w4.so w5:DPG_LIB_PATH=$L/libdpg_w5.so" bash tools/gpu_env_ab.sh
