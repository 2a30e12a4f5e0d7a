#!/bin/bash
# Streamed medium chunks (dpg_sortb.h tier 3): GPU suites touching them, the
# phase clocks of the (N = 1e9, U = 1e6) input, same-box A/Bs against the
# hash-table medium kernel (DPG_MEDIUM_STREAM=0) at (1e9, 1e6) and config 4.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r6h
if [ -z "$SKIP_TESTS" ]; then
TAG=r6h TESTS="tests/test_gpu_parity.py tests/test_gpu_envelope.py tests/test_gpu_configs.py" bash tools/gpu_check_ab.sh || exit 1
fi
DPG_PHASE_TIMING=1 timeout -k 10 300 python -u bench.py --records 1000000000 --pids 1000000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r6h/phase_u1e6.json 2> gpurun_out/r6h/phase_u1e6.err || { tail -5 gpurun_out/r6h/phase_u1e6.err; exit 1; }
grep "dpg phase" gpurun_out/r6h/phase_u1e6.err | tail -5
TAG=r6h/u1e6 STEPS=3 BENCH_ARGS="--records 1000000000 --pids 1000000" VARIANTS="stream:DPG_X=0 hash:DPG_MEDIUM_STREAM=0" bash tools/gpu_env_ab.sh || exit 1
TAG=r6h/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="stream:DPG_X=0 hash:DPG_MEDIUM_STREAM=0" bash tools/gpu_env_ab.sh || exit 1
