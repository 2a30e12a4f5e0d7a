#!/bin/bash
# Utility-analysis GPU tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ua.log 2>&1 || { echo pytest failed; grep -E "^E |Error|error" gpurun_out/pytest_ua.log | head -30; tail -5 gpurun_out/pytest_ua.log; exit 1; }
tail -3 gpurun_out/pytest_ua.log
