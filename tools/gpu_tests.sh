#!/bin/bash
# GPU tests of the given test files (default: all), then smoke.
# usage: bash tools/gpu_tests.sh [pytest paths...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
