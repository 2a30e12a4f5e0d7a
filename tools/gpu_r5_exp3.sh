#!/bin/bash
# Round-5 experiment 3: the piece-mode level-1 records per thread (A/B),
# then the whole GPU test suite and smoke on the product library.
set -o pipefail
export TMPDIR=/tmp
L=pipelinedp_amd/lib
TAG=r5e/ab VARIANTS="new:DPG_X=0 ipc9:DPG_LIB_PATH=$L/libdpg_ipc9.so ipc8:DPG_LIB_PATH=$L/libdpg_ipc8.so" bash tools/gpu_env_ab.sh || exit 1
mkdir -p gpurun_out/r5e
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5e/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED|Error" gpurun_out/r5e/pytest_gpu.log | head -30; tail -5 gpurun_out/r5e/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5e/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5e/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r5e/smoke.log; exit 1; }
tail -1 gpurun_out/r5e/smoke.log
