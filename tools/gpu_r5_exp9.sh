#!/bin/bash
# Round-5 experiment 9: k_ua_accumulate reading each pair's key, count and
# sum by scalar loads (28 instead of 31 VALU instructions per pair) -- the
# utility GPU tests, then same-box config-5 A/B against the LDS-broadcast
# build (h).
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_ua.log | head -20; tail -5 $O/pytest_ua.log; exit 1; }
tail -1 $O/pytest_ua.log
TAG=r5k/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="new:DPG_X=0 h:DPG_LIB_PATH=$L/libdpg_h.so" bash tools/gpu_env_ab.sh
