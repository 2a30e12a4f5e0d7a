#!/bin/bash
# Small-chunk packing cap (DPG_DEBUG_CAPS) at config 2, and the per-wave
# mcpp loop bound of the 2-wave kernel at config 4 (same-box A/Bs).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r6m
if [ -z "$SKIP_TESTS" ]; then
TAG=r6m TESTS="tests/test_gpu_parity.py" bash tools/gpu_check_ab.sh || exit 1
fi
TAG=r6m/c2 STEPS=4 VARIANTS="c512:DPG_X=0 c384:DPG_DEBUG_CAPS=384 c320:DPG_DEBUG_CAPS=320 c256:DPG_DEBUG_CAPS=256" bash tools/gpu_env_ab.sh || exit 1
TAG=r6m/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="c512:DPG_X=0 c384:DPG_DEBUG_CAPS=384" bash tools/gpu_env_ab.sh || exit 1
