#!/bin/bash
# Round-5 experiment 7: the pre-aggregate's two pair levels (items by
# partition-key range, pairs by the low key bits) in XCD-local mode
# (DPG_PA_XCD=1, DPG_PA_SUBS sub-tiles per tile) against the default
# tile-per-3072nd mode, config 5; rb10 = a 10 + 10 bit split of the key
# (DPG_PA_RB=10 build).  Parity first: the utility GPU tests with the switch on.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
mkdir -p gpurun_out/r5i
DPG_PA_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_utility.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5i/pytest_pa_xcd.log 2>&1 || { echo pytest failed; tail -20 gpurun_out/r5i/pytest_pa_xcd.log; exit 1; }
tail -1 gpurun_out/r5i/pytest_pa_xcd.log
TAG=r5i/ab STEPS=3 BENCH_ARGS="--workload config5" VARIANTS="base:DPG_PA_XCD=0 x4:DPG_PA_XCD=1,DPG_PA_SUBS=4 x1:DPG_PA_XCD=1,DPG_PA_SUBS=1 x16:DPG_PA_XCD=1,DPG_PA_SUBS=16 rb10:DPG_LIB_PATH=$L/libdpg_rb10.so" bash tools/gpu_env_ab.sh
