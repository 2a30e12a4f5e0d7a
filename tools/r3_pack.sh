#!/bin/bash
# packed-key narrow sort: parity, then same-box A/B vs DPG_SORT_PACKED=0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pack
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_release.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pack/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/pack/parity.log | head -30; tail -5 gpurun_out/pack/parity.log; exit 1; }
tail -1 gpurun_out/pack/parity.log
VARIANTS="libdpg_nopack.so" TAG=pk bash tools/gpu_ab.sh
