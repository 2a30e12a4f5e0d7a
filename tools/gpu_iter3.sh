#!/bin/bash
# parity tests of the partition / bounding kernels, then same-box A/B of the
# current library against $VARIANTS
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { echo pytest failed; grep -E "^E |FAILED|Error" gpurun_out/pytest_iter.log | head -20; tail -3 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
bash tools/gpu_ab.sh
