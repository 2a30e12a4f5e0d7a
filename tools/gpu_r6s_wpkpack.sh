#!/bin/bash
# Float64-packed wide partition keys in the single-wave sort passes: parity suites, then
# same-box A/B against the previous library at configs 4 and 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
T=r6s
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_release.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/$T/pytest.log | head -20; tail -5 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
TAG=$T/c4 STEPS=3 BENCH_ARGS="--workload config4" VARIANTS="npack:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
TAG=$T/c2 STEPS=5 VARIANTS="npack:DPG_X=0 base:DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_base.so" bash tools/gpu_env_ab.sh || exit 1
