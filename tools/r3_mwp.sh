#!/bin/bash
# packed-key multi-wave sort (variant lib): parity with the variant, then
# same-box config-4 A/B against the shipped library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mwp
DPG_LIB_PATH=pipelinedp_amd/lib/libdpg_mwp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/mwp/parity.log 2>&1 || { echo parity failed; grep -E "^E |FAILED|Error" gpurun_out/mwp/parity.log | head -30; tail -5 gpurun_out/mwp/parity.log; exit 1; }
tail -1 gpurun_out/mwp/parity.log
VARIANTS="libdpg_mwp.so" TAG=mwp BENCH_ARGS="--workload config4" bash tools/gpu_ab.sh
