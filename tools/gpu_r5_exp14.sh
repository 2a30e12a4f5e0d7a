#!/bin/bash
# Round-5 experiment 14: k_build_tiles with one wave per segment (the item
# level's single segment of ~3000 tiles was one thread's loop) -- partition
# parity tests on the variant, then same-box config-2 A/B.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5p
mkdir -p $O
DPG_LIB_PATH=$L/libdpg_tiles.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_utility.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=r5p/ab STEPS=10 VARIANTS="base:DPG_X=0 tiles:DPG_LIB_PATH=$L/libdpg_tiles.so" bash tools/gpu_env_ab.sh
