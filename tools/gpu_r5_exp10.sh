#!/bin/bash
# Round-5 experiment 10: k_ua_select split into an exact-PMF pass (<= 100
# pairs, 104-count keep table: more resident waves) and a normal-
# approximation pass, with the keep table sized by the last uncertain count
# -- utility GPU tests on the variant, then same-box config-5 A/B.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5l
mkdir -p $O
DPG_LIB_PATH=$L/libdpg_sel.so timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_ua.log | head -20; tail -5 $O/pytest_ua.log; exit 1; }
tail -1 $O/pytest_ua.log
TAG=r5l/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="base:DPG_X=0 sel:DPG_LIB_PATH=$L/libdpg_sel.so" bash tools/gpu_env_ab.sh
