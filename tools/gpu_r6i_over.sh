#!/bin/bash
# Oversize buckets streamed by the sort pass's tier 3 (DPG_STREAM_OVER): the
# GPU suites touching them, then same-box A/Bs against the heavy filter at
# (N = 1e9, U = 1e6) and config 4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r6i
if [ -z "$SKIP_TESTS" ]; then
TAG=r6i TESTS="tests/test_gpu_parity.py tests/test_gpu_envelope.py tests/test_gpu_configs.py" bash tools/gpu_check_ab.sh || exit 1
fi
TAG=r6i/u1e6 STEPS=3 BENCH_ARGS="--records 1000000000 --pids 1000000" VARIANTS="over:DPG_X=0 hvf:DPG_STREAM_OVER=0" bash tools/gpu_env_ab.sh || exit 1
TAG=r6i/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="over:DPG_X=0 hvf:DPG_STREAM_OVER=0" bash tools/gpu_env_ab.sh || exit 1
