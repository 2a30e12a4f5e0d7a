#!/bin/bash
# Round-5 experiment 17: the select kernel's normal-approximation pass with
# every class's moments loaded in one round and a 16-KB keep table (more
# resident waves) -- utility GPU tests, then same-box config-5 A/B against
# the previous build (base).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_ua.log | head -20; tail -5 $O/pytest_ua.log; exit 1; }
tail -1 $O/pytest_ua.log
TAG=r5s/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=$L/libdpg_base.so" bash tools/gpu_env_ab.sh
