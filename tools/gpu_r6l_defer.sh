#!/bin/bash
# Early deferral (BoundParams::defer_est): GPU suites, then same-box A/Bs of
# config 4 (early deferral on / off, a 23-bit plan) and config 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r6l
if [ -z "$SKIP_TESTS" ]; then
TAG=r6l TESTS="tests/test_gpu_parity.py tests/test_gpu_configs.py" bash tools/gpu_check_ab.sh || exit 1
fi
TAG=r6l/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="ed:DPG_X=0 noed:DPG_EARLY_DEFER=0 t128:DPG_DEBUG_TARGET=128" bash tools/gpu_env_ab.sh || exit 1
TAG=r6l/c2 STEPS=4 VARIANTS="ed:DPG_X=0 noed:DPG_EARLY_DEFER=0" bash tools/gpu_env_ab.sh || exit 1
