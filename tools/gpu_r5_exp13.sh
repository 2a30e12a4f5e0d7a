#!/bin/bash
# Round-5 experiment 13: the utility sweep without the 9.7 GB zero fill of
# its per-partition outputs (only rows of partitions split between
# accumulate runs are zeroed, k_ua_zero_split) -- utility GPU tests, then
# same-box config-5 A/B against the full fill (DPG_UA_FULL_ZERO=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED" $O/pytest_ua.log | head -20; tail -5 $O/pytest_ua.log; exit 1; }
tail -1 $O/pytest_ua.log
TAG=r5o/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="split:DPG_X=0 full:DPG_UA_FULL_ZERO=1" bash tools/gpu_env_ab.sh
