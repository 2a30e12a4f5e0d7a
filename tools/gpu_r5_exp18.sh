#!/bin/bash
# Round-5 experiment 18: the select kernel's telescoped upper mass computed
# for all classes in one pass (lane = class) -- utility GPU tests on the
# variant, then same-box config-5 A/B against the current build.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5t
mkdir -p $O
DPG_LIB_PATH=$L/libdpg_tele.so timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_ua.log | head -20; tail -5 $O/pytest_ua.log; exit 1; }
tail -1 $O/pytest_ua.log
TAG=r5t/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="cur:DPG_X=0 tele:DPG_LIB_PATH=$L/libdpg_tele.so" bash tools/gpu_env_ab.sh
