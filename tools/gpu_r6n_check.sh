#!/bin/bash
# Full GPU suite, then same-box A/B of config 4 and (1e9, 1e6) against the
# previous library (wave-aggregated chunk reservations, per-wave mcpp loop
# bound of the 2-wave kernel), and the config-2 line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=r6n
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/$T/pytest_gpu.log | head -20; tail -5 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$T/pytest_gpu.log
TAG=$T/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
TAG=$T/u1e6 STEPS=3 BENCH_ARGS="--records 1000000000 --pids 1000000" VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
TAG=$T/c2 STEPS=5 VARIANTS="new:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
