#!/bin/bash
# utility accumulate with compile-time metric flags (variant lib): utility /
# histogram parity with the variant, then same-box config-5 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/acci
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_acci.so timeout -k 10 600 python -u -m pytest tests/test_gpu_utility.py tests/test_gpu_histograms.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/acci/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/acci/parity.log | head -30; tail -5 gpurun_out/acci/parity.log; exit 1; }
tail -1 gpurun_out/acci/parity.log
timeout -k 10 300 python -u tools/ua_timing.py > gpurun_out/acci/base.log 2>&1 || { echo base failed; tail -5 gpurun_out/acci/base.log; exit 1; }
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_acci.so timeout -k 10 300 python -u tools/ua_timing.py > gpurun_out/acci/acc.log 2>&1 || { echo acc failed; tail -5 gpurun_out/acci/acc.log; exit 1; }
tail -n 1 gpurun_out/acci/base.log; tail -n 1 gpurun_out/acci/acc.log
